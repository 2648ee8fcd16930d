# round 6d: mask-only throughput -- one launch per B frames on ONE stream (B = 256 / 768 / 2048:
# the launch-level straggler tail paid once per B frames) vs 256-frame launches on 3 / 4 streams
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6d
timeout -k 10 300 python3 -u tools/bench_mask_overlap.py --batch 256 --streams 3,4,1 --launches 24 > gpurun_out/${T}_b256.log 2>&1 && echo B256_OK && \
timeout -k 10 300 python3 -u tools/bench_mask_overlap.py --batch 768 --streams 1,2 --launches 8 > gpurun_out/${T}_b768.log 2>&1 && echo B768_OK && \
timeout -k 10 300 python3 -u tools/bench_mask_overlap.py --batch 2048 --streams 1 --launches 3 > gpurun_out/${T}_b2048.log 2>&1 && echo B2048_OK
