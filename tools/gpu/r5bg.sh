# round 5bg: configs[2] chain with 512 / 128 solve threads per pair (one pair per launch) vs 256
set -o pipefail
mkdir -p gpurun_out
T=r5bg
L=$PWD/ssf-slam_amd/ssf/_lib
for rep in 1 2; do
for v in both nt512 nt128; do
  if [ $v = both ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 bench.py --consecutive 32 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_${v}_$rep.json 2> gpurun_out/${T}_${v}_$rep.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', round(d['value']), round(d['ms_per_step'],3))"
done
done
