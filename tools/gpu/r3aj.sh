# round 3aj (A): the final build -- every GPU test, the bench lines of every config
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3aj_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 400 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r3aj_bench.json 2> gpurun_out/r3aj_bench.err && echo BENCH_OK && \
timeout -k 10 300 python -u bench.py --latency --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r3aj_latency.json 2> gpurun_out/r3aj_latency.err && echo LAT_OK && \
timeout -k 10 300 python -u bench.py --consecutive 32 --batch 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3aj_consec.json 2> gpurun_out/r3aj_consec.err && echo CONSEC_OK && \
timeout -k 10 300 python -u bench.py --mask-before-features --batch 32 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3aj_c3.json 2> gpurun_out/r3aj_c3.err && echo C3_OK && \
timeout -k 10 400 python -u bench.py --n-az 4000 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3aj_c5.json 2> gpurun_out/r3aj_c5.err && echo C5_OK
