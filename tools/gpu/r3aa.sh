# round 3y: pass 0, GMM init and final pass with two points in flight
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mask.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3aa_pytest.log 2>&1 && echo PYTEST_OK && \
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r3aa_phases_b256.log 2>&1 && echo PH256_OK && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3aa_bench.log 2>&1 && echo BENCH_OK
