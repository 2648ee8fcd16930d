# round 5ak: k_solve compaction records per thread and pass 16 / 12 / 4 vs 8
set -o pipefail
mkdir -p gpurun_out
T=r5ak
L=$PWD/ssf-slam_amd/ssf/_lib
for rep in 1 2; do
for v in both cmp16 cmp12 cmp4; do
  if [ $v = both ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 tools/bench_features.py --reps 6 --chain > gpurun_out/${T}_${v}_$rep.json 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', d['kernel_ms']['k_solve'])"
done
done
