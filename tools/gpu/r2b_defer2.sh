set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
for n in frontend df3 df2m4 df2m3 df2r4 frontend; do f=libssf_frontend_$n.so; [ $n = frontend ] && f=libssf_frontend.so
SSF_LIB=$L/$f timeout -k 10 200 python -u tools/bench_features.py --chain --distinct 256 --reps 5 --tag $n >> gpurun_out/defer2.log 2>&1 || exit 1
SSF_LIB=$L/$f timeout -k 10 200 python -u tools/bench_features.py --chain --distinct 256 --reps 3 --n-az 4000 --tag ${n}_c5 >> gpurun_out/defer2.log 2>&1 || exit 1
done
