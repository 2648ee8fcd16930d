# round 6g: configs[2] as written (one sequence, 32 chained pairs per step) with the GN-specialised
# k_solve at 256 (default) vs 512 threads (s512), alternating
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6g
L=$PWD/ssf-slam_amd/ssf/_lib
for rep in 1 2; do
for v in def s512; do
  if [ $v = def ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 -u bench.py --consecutive 32 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_${v}_$rep.json 2> gpurun_out/${T}_${v}_$rep.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', round(d['value']), round(d['ms_per_step'],3))"
done
done
