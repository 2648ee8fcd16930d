# round 6a: per-step serial cost along the sequences (diag_mask_window) + the default line at
# warmup 5 / 50 on one box (name the late-window drop)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6a
timeout -k 10 300 python -u tools/diag_mask_window.py gpurun_out/${T}_window.json 150 > gpurun_out/${T}_window.log 2>&1 && echo WIN_OK && \
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_w5.json 2> gpurun_out/${T}_w5.err && echo W5_OK && \
timeout -k 10 300 python -u bench.py --steps 40 --warmup 60 --no-cpu-baseline > gpurun_out/${T}_w60.json 2> gpurun_out/${T}_w60.err && echo W60_OK
