# round 4aq: configs[2] / configs[3] lines with the default 5 warmup steps (the caching allocator and
# the mask's draw-slot ring reach their steady state in ~3 steps; 1-2 warmup steps left host
# stalls of 7-60 ms in the first timed steps, r4ap)
set -o pipefail
mkdir -p gpurun_out
T=r4aq
NB="--no-cpu-baseline"
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 7 --warmup 5 $NB --timeline > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4.err && echo C4 && \
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 7 --warmup 5 --kabsch-warm-start $NB > gpurun_out/${T}_c4kws.json 2> gpurun_out/${T}_c4kws.err && echo C4KWS && \
timeout -k 10 300 python -u bench.py --consecutive 32 --steps 10 --warmup 5 $NB > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err && echo C3 && \
timeout -k 10 300 python -u bench.py --consecutive 32 --steps 10 --warmup 5 --kabsch-warm-start $NB --timeline > gpurun_out/${T}_c3kws.json 2> gpurun_out/${T}_c3kws.err && echo C3KWS && \
timeout -k 10 400 python -u bench.py --gpus 2 --sequences-total 8 --consecutive 32 --steps 7 --warmup 5 --rehearse-one-gpu $NB > gpurun_out/${T}_c4n2.json 2> gpurun_out/${T}_c4n2.err && echo C4N2
