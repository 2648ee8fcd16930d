# round 5ao: the carla bench line's k_feat_wave_run (HIP events, kernel pass): default (4 registers
# in flight) vs 3, vs 3 + the one-ballot interior test; alternating
set -o pipefail
mkdir -p gpurun_out
T=r5ao
L=$PWD/ssf-slam_amd/ssf/_lib
for rep in 1 2 3; do
for v in both pf3 pf3b1; do
  if [ $v = both ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 bench.py --layout carla --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_${v}_$rep.json 2> gpurun_out/${T}_${v}_$rep.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$rep.json').read().strip().splitlines()[-1]);k=d['kernels']['k_feat_wave_run'];print('$v', round(k['ms'],4), round(k['frac'],4), round(d['value']))"
done
done
