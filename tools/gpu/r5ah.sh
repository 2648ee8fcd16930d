# round 5ah: same-box A/B of the default line, session-start build (tmp_base, e541ad8) vs HEAD
set -o pipefail
mkdir -p gpurun_out
T=r5ah
R=$PWD
for rep in 1 2; do
for v in base head; do
  if [ $v = base ]; then d=$R/tmp_base; else d=$R; fi
  (cd $d && timeout -k 10 600 python -u bench.py --no-cpu-baseline --steps 60 > $R/gpurun_out/${T}_${v}_$rep.json 2> $R/gpurun_out/${T}_${v}_$rep.err) || { echo "${v}_FAIL"; tail -5 $R/gpurun_out/${T}_${v}_$rep.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$R/gpurun_out/${T}_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', round(d['value']), round(d['ms_per_step'],3))"
done
done
