# round 4au: configs[2] with Kabsch warm starts -- mask split and mask streams (proper warmup)
set -o pipefail
mkdir -p gpurun_out
T=r4au
K="python -u bench.py --consecutive 32 --kabsch-warm-start --steps 10 --warmup 5 --no-cpu-baseline"
timeout -k 10 200 $K > gpurun_out/${T}_auto.json 2>/dev/null && echo a && \
timeout -k 10 200 $K --mask-split 4 > gpurun_out/${T}_g4.json 2>/dev/null && echo b && \
timeout -k 10 200 $K --mask-split 2 > gpurun_out/${T}_g2.json 2>/dev/null && echo c && \
timeout -k 10 200 $K --mask-streams 2 > gpurun_out/${T}_s2.json 2>/dev/null && echo d && \
timeout -k 10 200 $K --mask-streams 4 > gpurun_out/${T}_s4.json 2>/dev/null && echo e && \
timeout -k 10 200 $K --mask-split 4 --mask-streams 4 > gpurun_out/${T}_g4s4.json 2>/dev/null && echo f && \
timeout -k 10 200 $K --steps 30 > gpurun_out/${T}_auto30.json 2>/dev/null && echo g
