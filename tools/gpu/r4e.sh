# round 4e: the single-read feature stage -- parity tests, then kernel times against the legacy
# four-kernel stage (same box, alternating)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_configs.py tests/test_gpu_edges.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4e_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 120 python -u tools/bench_features.py --reps 5 > gpurun_out/r4e_new1.json 2>&1 && \
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_legacy.so timeout -k 10 120 python -u tools/bench_features.py --reps 5 > gpurun_out/r4e_old1.json 2>&1 && \
timeout -k 10 120 python -u tools/bench_features.py --reps 5 > gpurun_out/r4e_new2.json 2>&1 && \
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_legacy.so timeout -k 10 120 python -u tools/bench_features.py --reps 5 > gpurun_out/r4e_old2.json 2>&1 && echo BENCH_OK
