# round 4be: association with at least 2 / 3 work-groups per pair at B = 256
set -o pipefail
mkdir -p gpurun_out
T=r4be
L=$PWD/ssf-slam_amd/ssf/_lib
for i in 1 2; do
  for v in default as2 as3; do
    if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
    SSF_LIB=$lib timeout -k 10 120 python -u tools/bench_features.py --reps 5 --chain --distinct 32 --tag $v > gpurun_out/${T}_${v}_$i.json 2>&1 || exit 1
  done
done
for v in default as2; do
  if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_def_$v.json 2>/dev/null || exit 1
done
echo ALL_OK
