set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --edges --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r2v_bench_edges.log 2>&1 && echo EDGES_OK && \
timeout -k 10 300 python -u bench.py --edges --serial --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/r2v_bench_edges_serial.log 2>&1 && echo EDGES_SERIAL_OK
