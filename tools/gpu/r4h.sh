# round 4h: why configs[3] / configs[2] steps take longer than the default bench's -- kernel stats of
# the strong-scaling mode, and the mask split / stream settings for many frames per step
set -o pipefail
mkdir -p gpurun_out
R=$PWD
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4h_prof -o p -- python3 $R/bench.py --sequences-total 8 --consecutive 32 --steps 4 --warmup 1 --kabsch-warm-start --no-cpu-baseline > $R/gpurun_out/r4h_c4_prof.json 2> $R/gpurun_out/r4h_c4_prof.err ) && echo PROF_OK && \
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 7 --warmup 1 --kabsch-warm-start --mask-streams 6 --no-cpu-baseline > gpurun_out/r4h_c4_kws_ms6.json 2> gpurun_out/r4h_c4_kws_ms6.err && echo C4MS6_OK && \
timeout -k 10 300 python -u bench.py --consecutive 32 --steps 10 --warmup 2 --kabsch-warm-start --mask-split 1 --mask-streams 8 --no-cpu-baseline > gpurun_out/r4h_c3_kws_g1.json 2> gpurun_out/r4h_c3_kws_g1.err && echo C3G1_OK
