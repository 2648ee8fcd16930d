set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_edges.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2w_edges.log 2>&1 && echo EDGES_TESTS_OK && \
timeout -k 10 300 python -u bench.py --edges --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r2w_bench_edges.log 2>&1 && echo EDGES_OK
