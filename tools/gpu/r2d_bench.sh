set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2d_bench.log 2>&1 && echo BENCH_OK && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --n-az 4000 > gpurun_out/r2d_c5.log 2>&1 && echo C5_OK && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --mask-before-features --batch 32 > gpurun_out/r2d_c3.log 2>&1 && echo C3_OK
