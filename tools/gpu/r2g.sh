set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r2g_gpu_tests.log 2>&1 && echo TESTS_OK && \
timeout -k 10 300 python -u bench.py --mask-before-features --batch 32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r2g_bench_c3.log 2>&1 && echo BENCH3_OK
