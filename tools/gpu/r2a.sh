set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2a_gpu_tests.log 2>&1 && echo TESTS_OK && \
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r2a_smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 240 python -u bench.py > gpurun_out/r2a_bench.log 2>&1 && echo BENCH_OK
