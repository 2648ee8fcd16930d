set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/tail20.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline --kernel-pass 0 > gpurun_out/tail60.log 2>&1
