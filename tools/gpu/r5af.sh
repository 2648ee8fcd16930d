# round 5af: k_solve A/B: 512 threads per pair (2 waves per SIMD), correspondences per step 4 / 1
set -o pipefail
mkdir -p gpurun_out
T=r5af
L=$PWD/ssf-slam_amd/ssf/_lib
for rep in 1 2; do
for v in both nt512 step4 step1; do
  if [ $v = both ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 tools/bench_features.py --reps 6 --chain > gpurun_out/${T}_${v}_$rep.json 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', d['kernel_ms']['k_solve'])"
done
done
