# round 3ah: radius doubling in the plane table's deferred filtered 1-NN
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3ah_pytest.log 2>&1 && echo PYTEST_OK && \
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_table_phases.py 256 > gpurun_out/r3ah_table.log 2>&1 && echo T_OK && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-pass 5 > gpurun_out/r3ah_bench.log 2>&1 && echo BENCH_OK
