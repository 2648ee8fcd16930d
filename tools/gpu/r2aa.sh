set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py tests/test_gpu_nodes.py tests/test_examples.py tests/test_gpu_edges.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2aa_tests.log 2>&1 && echo TESTS_OK && \
timeout -k 10 400 python -u bench.py --n-az 4000 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r2aa_bench_c5.log 2>&1 && echo BENCH5_OK
