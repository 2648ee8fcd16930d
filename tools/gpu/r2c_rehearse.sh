set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u bench.py --gpus 2 --rehearse-one-gpu --steps 5 --warmup 2 --batch 64 --no-cpu-baseline --kernel-pass 0 > gpurun_out/r2c_rehearse.log 2>&1
