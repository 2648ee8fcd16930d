set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_sstamp.so timeout -k 10 200 python -u tools/bench_features.py --chain --stamps --reps 5 --tag sstamp > gpurun_out/r2c_solve.log 2>&1 && echo SOLVE_OK
