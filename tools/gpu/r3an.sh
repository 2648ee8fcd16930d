# round 3an: smoke() and a short default bench of the final tree (the line carries the r03ak traffic)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_DONE')" > gpurun_out/r3an_smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3an_bench.log 2>&1 && echo BENCH_OK
