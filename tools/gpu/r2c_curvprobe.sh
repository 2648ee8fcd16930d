set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
for n in frontend cp1 cp1d6 cp2 cp2r1 frontend; do f=libssf_frontend_$n.so; [ $n = frontend ] && f=libssf_frontend.so; SSF_LIB=$L/$f timeout -k 10 200 python -u tools/bench_features.py --tag $n --reps 10 >> gpurun_out/r2c_curvprobe.log 2>&1 || exit 1; done && echo PROBE_OK
