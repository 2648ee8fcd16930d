# round 3w: EM skip passes (state bytes, open-point and set-1-change queues)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mask.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3w_pytest.log 2>&1 && echo PYTEST_OK && \
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r3w_phases_b256.log 2>&1 && echo PH256_OK && \
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_mask_phases.py 1 > gpurun_out/r3w_phases_b1.log 2>&1 && echo PH1_OK && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3w_bench.log 2>&1 && echo BENCH_OK
