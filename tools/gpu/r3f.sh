# round 3f: state check after the container re-creation -- full GPU suite, smoke, the no-flag
# bench line (CPU legs included), the configs[1] latency line, configs[2] as written, and a
# rocprof kernel-trace of the serial kernel pass
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3f_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3f_smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 400 python -u bench.py > gpurun_out/r3f_bench.json 2> gpurun_out/r3f_bench.err && echo BENCH_OK && \
timeout -k 10 200 python -u bench.py --latency --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r3f_lat.json 2> gpurun_out/r3f_lat.err && echo LAT_OK && \
timeout -k 10 300 python -u bench.py --consecutive 32 --batch 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3f_consec.json 2> gpurun_out/r3f_consec.err && echo CONSEC_OK && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3f_prof_serial -o serial -- python3 bench.py --serial --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3f_prof_serial.log 2>&1 && echo PROF_OK
