# round 6i: mask-only throughput with the frame queue (192 / 160 work-groups per launch) vs one
# work-group per frame, 256-frame launches on 2 / 3 streams; then the default bench (queue 192)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6i
timeout -k 10 300 python3 -u tools/bench_mask_overlap.py --batch 256 --streams 3,2 --launches 30 > gpurun_out/${T}_q0.log 2>&1 && echo Q0_OK && \
timeout -k 10 300 python3 -u tools/bench_mask_overlap.py --batch 256 --streams 3,2,1 --launches 30 --queue 192 > gpurun_out/${T}_q192.log 2>&1 && echo Q192_OK && \
timeout -k 10 300 python3 -u tools/bench_mask_overlap.py --batch 256 --streams 3 --launches 30 --queue 160 > gpurun_out/${T}_q160.log 2>&1 && echo Q160_OK && \
timeout -k 10 300 python3 -u bench.py --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_default.json 2> gpurun_out/${T}_default.err && echo DEF_OK
