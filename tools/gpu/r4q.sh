# round 4q: configs[2] (one sequence, 32 chained pairs per step): current build vs the r04b build,
# and the mask-stream / mask-split knobs
set -o pipefail
mkdir -p gpurun_out
T=r4q
NB="--no-cpu-baseline"
C3="python -u bench.py --consecutive 32 --steps 10 --warmup 2 $NB"
L=$GRAFT_REPO_ROOT/ssf-slam_amd/ssf/_lib
timeout -k 10 200 $C3 > gpurun_out/${T}_cur.json 2> gpurun_out/${T}_cur.err && echo A && \
SSF_LIB=$L/libssf_frontend_r04b.so timeout -k 10 200 $C3 > gpurun_out/${T}_r04b.json 2> gpurun_out/${T}_r04b.err && echo B && \
timeout -k 10 200 $C3 > gpurun_out/${T}_cur2.json 2> gpurun_out/${T}_cur2.err && echo C && \
SSF_LIB=$L/libssf_frontend_r04b.so timeout -k 10 200 $C3 > gpurun_out/${T}_r04b2.json 2> gpurun_out/${T}_r04b2.err && echo D && \
timeout -k 10 200 $C3 --mask-streams 1 > gpurun_out/${T}_cur_ms1.json 2> gpurun_out/${T}_cur_ms1.err && echo E && \
timeout -k 10 200 $C3 --mask-split 4 > gpurun_out/${T}_cur_g4.json 2> gpurun_out/${T}_cur_g4.err && echo F && \
SSF_LIB=$L/libssf_frontend_legacy.so timeout -k 10 200 $C3 > gpurun_out/${T}_legacy.json 2> gpurun_out/${T}_legacy.err && echo G
