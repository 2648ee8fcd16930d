# round 4bn: the mask alone, B = 256 launches over 1-4 streams (the pipeline's ceiling if the
# chain cost nothing), beside the default line on the same box
set -o pipefail
mkdir -p gpurun_out
T=r4bn
timeout -k 10 300 python -u tools/bench_mask_overlap.py --streams 1,2,3,4 --launches 30 > gpurun_out/${T}_mask_overlap.json 2> gpurun_out/${T}_mask_overlap.err && echo MASK && \
timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_def.json 2> gpurun_out/${T}_def.err && echo DEF
