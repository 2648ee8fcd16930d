set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b2_default.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --n-az 4000 > gpurun_out/b2_c5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --mask-before-features --batch 32 > gpurun_out/b2_c3.log 2>&1
