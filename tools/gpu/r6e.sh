# round 6e: frame order within a mask launch (tools/diag_mask_order.py): sequence order vs
# longest-first by the previous step's cost vs by the frames' own cost; 3-stream throughput
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6e
timeout -k 10 400 python3 -u tools/diag_mask_order.py gpurun_out/${T}_order.json 12 > gpurun_out/${T}_order.log 2>&1 && echo ORDER_OK
