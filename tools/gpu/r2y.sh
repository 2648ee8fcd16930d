set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mask.py tests/test_gpu_configs.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r2y_mask_tests.log 2>&1 && echo MASK_TESTS_OK && \
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r2y_phases.log 2>&1 && echo PHASES_OK && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2y_bench.log 2>&1 && echo BENCH_OK
