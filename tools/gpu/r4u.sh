# round 4u: where k_feat_chunk's time goes -- timing variants that stop after phase 1..4
# (ring ids / + ranking and row scan / + place / + stencils; tools-only builds, no select)
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
for i in 1 2; do
  for v in default cut1 cut2 cut3 cut4; do
    if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
    SSF_LIB=$lib timeout -k 10 120 python -u tools/bench_features.py --reps 5 --tag $v > gpurun_out/r4u_${v}_$i.json 2>&1 || exit 1
  done
done
echo ALL_OK
