# round 4ao: configs[3] as written (8 sequences, 32 consecutive frames per step) -- per-step
# stream timelines, chained and Kabsch warm starts
set -o pipefail
mkdir -p gpurun_out
T=r4ao
C="python -u bench.py --sequences-total 8 --consecutive 32 --steps 6 --warmup 1 --no-cpu-baseline --timeline"
timeout -k 10 300 $C > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4.err && echo A && \
timeout -k 10 300 $C --kabsch-warm-start > gpurun_out/${T}_c4kws.json 2> gpurun_out/${T}_c4kws.err && echo B
