set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r2c_gpu_tests.log 2>&1 && echo TESTS_OK && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2c_smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2c_bench.log 2>&1 && echo BENCH_OK
