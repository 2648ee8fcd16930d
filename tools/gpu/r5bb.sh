# round 5bb: k_feat_select work-group size 512 / 256 vs 1024
set -o pipefail
mkdir -p gpurun_out
T=r5bb
L=$PWD/ssf-slam_amd/ssf/_lib
for rep in 1 2; do
for v in both s512 s256; do
  if [ $v = both ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 tools/bench_features.py --reps 8 > gpurun_out/${T}_${v}_$rep.json 2>&1 || exit 1
  SSF_LIB=$lib timeout -k 10 300 python3 tools/bench_features.py --reps 8 --layout carla > gpurun_out/${T}_${v}_c$rep.json 2>&1 || exit 1
  python3 -c "import json;a=json.loads(open('gpurun_out/${T}_${v}_$rep.json').read().strip().splitlines()[-1]);b=json.loads(open('gpurun_out/${T}_${v}_c$rep.json').read().strip().splitlines()[-1]);print('$v', a['kernel_ms']['k_feat_select'], b['kernel_ms']['k_feat_select'])"
done
done
