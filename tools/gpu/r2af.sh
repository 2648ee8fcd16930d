set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
for n in frontend d2r4 d4r4 d3r2 d3r8 d3r16; do f=libssf_frontend_$n.so; [ $n = frontend ] && f=libssf_frontend.so; SSF_LIB=$L/$f timeout -k 10 200 python -u tools/bench_features.py --tag $n --reps 5 >> gpurun_out/r2af_curv.log 2>&1 || exit 1; done && echo AB_OK
