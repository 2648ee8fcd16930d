# round 3r: the N > 1 path of bench.py rehearsed on one GPU (2 ranks, gloo, deferred pose
# all-gather) -- the driver runs N = 2 / 4 / 8 on an 8-GPU node at round end
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u bench.py --gpus 2 --rehearse-one-gpu --steps 10 --warmup 2 --batch 64 --no-cpu-baseline --kernel-pass 0 > gpurun_out/r3r_rehearse.log 2>&1 && echo REHEARSE_OK
