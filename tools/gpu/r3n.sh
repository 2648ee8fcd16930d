# round 3n: association split over up to 8 work-groups per pair for small launches (mask kernel
# as committed): GPU suite, default bench, latency, configs[2] both forms
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3n_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 400 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r3n_bench.json 2> gpurun_out/r3n_bench.err && echo BENCH_OK && \
timeout -k 10 200 python -u bench.py --latency --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r3n_lat.json 2> gpurun_out/r3n_lat.err && echo LAT_OK && \
timeout -k 10 300 python -u bench.py --consecutive 32 --batch 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3n_consec.json 2> gpurun_out/r3n_consec.err && echo CONSEC_OK && \
timeout -k 10 300 python -u bench.py --mask-before-features --batch 32 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3n_c3.json 2> gpurun_out/r3n_c3.err && echo C3_OK
