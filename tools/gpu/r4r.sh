# round 4r: the default bench (configs[1], 256 frames per mask launch) with fixed mask splits and
# mask-stream counts, one box
set -o pipefail
mkdir -p gpurun_out
T=r4r
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline"
timeout -k 10 200 $B > gpurun_out/${T}_g1.json 2> gpurun_out/${T}_g1.err && echo g1 && \
timeout -k 10 200 $B --mask-split 2 > gpurun_out/${T}_g2.json 2> gpurun_out/${T}_g2.err && echo g2 && \
timeout -k 10 200 $B --mask-split 4 > gpurun_out/${T}_g4.json 2> gpurun_out/${T}_g4.err && echo g4 && \
timeout -k 10 200 $B --mask-split 2 --mask-streams 2 > gpurun_out/${T}_g2s2.json 2> gpurun_out/${T}_g2s2.err && echo g2s2 && \
timeout -k 10 200 $B --mask-split 4 --mask-streams 2 > gpurun_out/${T}_g4s2.json 2> gpurun_out/${T}_g4s2.err && echo g4s2 && \
timeout -k 10 200 $B --mask-streams 4 > gpurun_out/${T}_g1s4.json 2> gpurun_out/${T}_g1s4.err && echo g1s4 && \
timeout -k 10 200 $B > gpurun_out/${T}_g1b.json 2> gpurun_out/${T}_g1b.err && echo g1b
