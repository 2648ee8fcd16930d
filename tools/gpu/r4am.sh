# round 4am: k_feat_chunk_reg occupancy -- y / z halo columns one coordinate ahead at 6 / 7 / 8
# waves per SIMD, and the default at 6, against the default (5 waves)
set -o pipefail
mkdir -p gpurun_out
T=r4am
L=$PWD/ssf-slam_amd/ssf/_lib
for i in 1 2; do
  for v in default s6 s7 s8 w6; do
    if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
    SSF_LIB=$lib timeout -k 10 120 python -u tools/bench_features.py --reps 5 --tag $v > gpurun_out/${T}_${v}_$i.json 2>&1 || exit 1
  done
done
echo ALL_OK
