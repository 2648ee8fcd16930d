set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mask.py tests/test_gpu_configs.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r2m_mask_tests.log 2>&1 && echo MASKTESTS_OK && \
timeout -k 10 200 python -u tools/bench_mask.py --batch 32 --splits 1,2,4,8 > gpurun_out/r2m_mask.log 2>&1 && echo B32_OK && \
timeout -k 10 200 python -u tools/bench_mask.py --batch 256 --splits 1,2 --distinct 64 >> gpurun_out/r2m_mask.log 2>&1 && echo B256_OK
