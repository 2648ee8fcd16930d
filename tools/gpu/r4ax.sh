# round 4ax: k_solve at 256 / 512 / 1024 threads per pair (bench_features --chain)
set -o pipefail
mkdir -p gpurun_out
T=r4ax
L=$PWD/ssf-slam_amd/ssf/_lib
for i in 1 2; do
  for v in default sv512 sv1024; do
    if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
    SSF_LIB=$lib timeout -k 10 120 python -u tools/bench_features.py --reps 5 --chain --tag $v > gpurun_out/${T}_${v}_$i.json 2>&1 || exit 1
  done
done
echo ALL_OK
