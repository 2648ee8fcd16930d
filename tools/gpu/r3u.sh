# round 3u: the association stages the plane table's strip image instead of rebuilding it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3u_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python -u bench.py --latency --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r3u_latency.log 2>&1 && echo LAT_OK && \
timeout -k 10 300 python -u bench.py --consecutive 32 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r3u_consec.log 2>&1 && echo CONSEC_OK && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3u_bench.log 2>&1 && echo BENCH_OK
