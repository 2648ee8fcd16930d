# round 4bl: the --f64-inputs line ran at 185 ms per step in r4bk (33.4 k frames/s = 7.7 ms in
# r04bc): repeat it, with per-step stream timelines, on the final build and on the build with
# k_feat_chunk_reg (variant chunkreg)
set -o pipefail
mkdir -p gpurun_out
T=r4bl
L=$GRAFT_REPO_ROOT/ssf-slam_amd/ssf/_lib
NB="--no-cpu-baseline"
timeout -k 10 300 python -u bench.py --f64-inputs --steps 20 --warmup 3 $NB > gpurun_out/${T}_f64in_1.json 2> gpurun_out/${T}_f64in_1.err && echo A && \
timeout -k 10 300 python -u bench.py --f64-inputs --steps 20 --warmup 3 --timeline $NB > gpurun_out/${T}_f64in_tl.json 2> gpurun_out/${T}_f64in_tl.err && echo B && \
SSF_LIB=$L/libssf_frontend_chunkreg.so timeout -k 10 300 python -u bench.py --f64-inputs --steps 20 --warmup 3 $NB > gpurun_out/${T}_f64in_chunkreg.json 2> gpurun_out/${T}_f64in_chunkreg.err && echo C
