# round 4y: configs[2] with Kabsch warm starts -- per-step stream timelines (HIP events), automatic
# split vs G = 1 over 4 mask streams
set -o pipefail
mkdir -p gpurun_out
K="python -u bench.py --consecutive 32 --kabsch-warm-start --steps 8 --warmup 2 --no-cpu-baseline --timeline"
timeout -k 10 200 $K > gpurun_out/r4y_auto.json 2> gpurun_out/r4y_auto.err && echo A && \
timeout -k 10 200 $K --mask-split 1 --mask-streams 4 > gpurun_out/r4y_g1s4.json 2> gpurun_out/r4y_g1s4.err && echo B && \
timeout -k 10 200 $K --mask-streams 1 > gpurun_out/r4y_s1.json 2> gpurun_out/r4y_s1.err && echo C
