# round 4ad: where k_feat_select's time goes -- timing variants stopping after phase 1..4
# (row bases / + plane transposition / + unresolved points / + greedy), on the g5 feature build
set -o pipefail
mkdir -p gpurun_out
T=r4ad
L=$PWD/ssf-slam_amd/ssf/_lib
for i in 1 2; do
  for v in g5 sc1 sc2 sc3 sc4; do
    SSF_LIB=$L/libssf_frontend_$v.so timeout -k 10 120 python -u tools/bench_features.py --reps 5 --tag $v > gpurun_out/${T}_${v}_$i.json 2>&1 || exit 1
  done
done
echo ALL_OK
