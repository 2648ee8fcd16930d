# round 5ac: plane table deferred-query group size 8 / 4 / 2
set -o pipefail
mkdir -p gpurun_out
T=r5ac
L=$PWD/ssf-slam_amd/ssf/_lib
echo skip-tests
for rep in 1 2; do
for v in tcoop8 tcoop4 tcoop2; do
  if [ $v = both ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 tools/bench_features.py --reps 6 --chain > gpurun_out/${T}_${v}_$rep.json 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', d['kernel_ms']['k_plane_table_sorted'])"
done
done
