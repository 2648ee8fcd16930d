# round 6zi: mask queue re-swept on the final build (60 steps, warmup 5), alternating
#
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6zi
for rep in 1 2; do
for cfg in "q-1:--mask-queue -1" "q176:--mask-queue 176" "q208:--mask-queue 208" "q224:--mask-queue 224"; do
  name=${cfg%%:*}; fl=${cfg#*:}
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline $fl > gpurun_out/${T}_${name}_$rep.json 2> gpurun_out/${T}_${name}_$rep.err || { tail -5 gpurun_out/${T}_${name}_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['config'].get('mask_schedule'))" gpurun_out/${T}_${name}_$rep.json $name
done
done
