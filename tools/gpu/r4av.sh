# round 4av: configs[2] lines at 30 timed steps (steady state), split knobs
set -o pipefail
mkdir -p gpurun_out
T=r4av
K="python -u bench.py --consecutive 32 --steps 30 --warmup 5 --no-cpu-baseline"
timeout -k 10 200 $K > gpurun_out/${T}_c3.json 2>/dev/null && echo a && \
timeout -k 10 200 $K --kabsch-warm-start > gpurun_out/${T}_kws.json 2>/dev/null && echo b && \
timeout -k 10 200 $K --kabsch-warm-start --mask-split 2 > gpurun_out/${T}_kws_g2.json 2>/dev/null && echo c && \
timeout -k 10 200 $K --kabsch-warm-start --mask-split 4 --mask-streams 4 > gpurun_out/${T}_kws_g4s4.json 2>/dev/null && echo d && \
timeout -k 10 200 $K --mask-split 2 > gpurun_out/${T}_c3_g2.json 2>/dev/null && echo e && \
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 12 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_c4.json 2>/dev/null && echo f && \
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 12 --warmup 5 --kabsch-warm-start --no-cpu-baseline > gpurun_out/${T}_c4kws.json 2>/dev/null && echo g
