# round 3a: GPU suite (incl. the multi-ticket split test), the configs[1] latency line, the
# default bench with the GPU data generator, a rocprof summary of the latency run
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3a_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python -u bench.py --latency --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r3a_latency.json 2> gpurun_out/r3a_latency.err && echo LATENCY_OK && \
timeout -k 10 400 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r3a_bench.json 2> gpurun_out/r3a_bench.err && echo BENCH_OK && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3a_prof_lat -o lat -- python3 bench.py --latency --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3a_prof_lat.log 2>&1 && echo PROF_OK
