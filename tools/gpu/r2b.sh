set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2b_gpu_tests.log 2>&1 && echo TESTS_OK && \
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r2b_bench.log 2>&1 && echo BENCH_OK && \
timeout -k 10 300 python -u bench.py --n-az 4000 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r2b_bench_c5.log 2>&1 && echo BENCH5_OK && \
timeout -k 10 300 python -u bench.py --mask-before-features --batch 32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r2b_bench_c3.log 2>&1 && echo BENCH3_OK
