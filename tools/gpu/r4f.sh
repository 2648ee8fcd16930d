# round 4f: single-read stage with the ring-id table + ring-order select; strip-image validity --
# parity tests, kernel times vs legacy
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_registration.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4f_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 120 python -u tools/bench_features.py --reps 5 > gpurun_out/r4f_new1.json 2>&1 && \
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_legacy.so timeout -k 10 120 python -u tools/bench_features.py --reps 5 > gpurun_out/r4f_old1.json 2>&1 && \
timeout -k 10 120 python -u tools/bench_features.py --reps 5 > gpurun_out/r4f_new2.json 2>&1 && echo BENCH_OK
