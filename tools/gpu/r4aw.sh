# round 4aw: configs[2] / configs[3] lines with the stream-aware mask split (slots / (streams x frames))
set -o pipefail
mkdir -p gpurun_out
T=r4aw
K="python -u bench.py --consecutive 32 --steps 30 --warmup 5 --no-cpu-baseline"
timeout -k 10 200 $K > gpurun_out/${T}_c3.json 2>/dev/null && echo a && \
timeout -k 10 200 $K --kabsch-warm-start > gpurun_out/${T}_c3kws.json 2>/dev/null && echo b && \
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 12 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_c4.json 2>/dev/null && echo c && \
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 12 --warmup 5 --kabsch-warm-start --no-cpu-baseline > gpurun_out/${T}_c4kws.json 2>/dev/null && echo d && \
timeout -k 10 400 python -u bench.py --gpus 2 --sequences-total 8 --consecutive 32 --steps 12 --warmup 5 --rehearse-one-gpu --no-cpu-baseline > gpurun_out/${T}_c4n2.json 2>/dev/null && echo e
