# round 4s: hardware queues (GPU_MAX_HW_QUEUES) x mask streams x split, default bench and configs[2] kws
set -o pipefail
mkdir -p gpurun_out
T=r4s
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline"
K="python -u bench.py --consecutive 32 --kabsch-warm-start --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 200 $B > gpurun_out/${T}_def_q4.json 2> gpurun_out/${T}_def_q4.err && echo a && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $B > gpurun_out/${T}_def_q8.json 2> gpurun_out/${T}_def_q8.err && echo b && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $B --mask-streams 5 > gpurun_out/${T}_def_q8s5.json 2> gpurun_out/${T}_def_q8s5.err && echo c && \
timeout -k 10 200 $K > gpurun_out/${T}_kws_q4.json 2> gpurun_out/${T}_kws_q4.err && echo d && \
timeout -k 10 200 $K --mask-split 1 > gpurun_out/${T}_kws_q4_g1.json 2> gpurun_out/${T}_kws_q4_g1.err && echo e && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $K > gpurun_out/${T}_kws_q8.json 2> gpurun_out/${T}_kws_q8.err && echo f && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $K --mask-split 1 --mask-streams 6 > gpurun_out/${T}_kws_q8_g1s6.json 2> gpurun_out/${T}_kws_q8_g1s6.err && echo g && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $K --mask-split 2 --mask-streams 6 > gpurun_out/${T}_kws_q8_g2s6.json 2> gpurun_out/${T}_kws_q8_g2s6.err && echo h && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $K --mask-split 4 --mask-streams 6 > gpurun_out/${T}_kws_q8_g4s6.json 2> gpurun_out/${T}_kws_q8_g4s6.err && echo i
