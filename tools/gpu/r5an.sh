# round 5an: k_feat_wave_run on carla frames: scalar load offset / one-ballot interior test /
# 6 or 10 waves per SIMD / 3 registers in flight, vs the default
set -o pipefail
mkdir -p gpurun_out
T=r5an
L=$PWD/ssf-slam_amd/ssf/_lib
for rep in 1 2 3; do
for v in both soff ball1 w6 w10 pf3; do
  if [ $v = both ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 tools/bench_features.py --reps 8 --layout carla > gpurun_out/${T}_${v}_$rep.json 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', d['kernel_ms']['k_feat_wave_run'])"
done
done
