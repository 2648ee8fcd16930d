set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_ctwice.so timeout -k 10 200 python -u tools/bench_features.py --tag twice --reps 10 > gpurun_out/r2c_twice.log 2>&1 && echo TWICE_OK || exit 1
for n in frontend bc2048 frontend bc2048; do f=libssf_frontend_$n.so; [ $n = frontend ] && f=libssf_frontend.so; echo $n >> gpurun_out/r2c_bc.log; SSF_LIB=$L/$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/r2c_bc.log 2>&1 || exit 1; done && echo BC_OK
