# round 5a: every GPU test (ring-id chains, the plane-table share fix), smoke, a default bench line
set -o pipefail
mkdir -p gpurun_out
T=r5a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_default.json 2> gpurun_out/${T}_default.err && echo BENCH_OK
