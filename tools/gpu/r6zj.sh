# round 6zj: mask queue 192 / 176 / 160 on the final build, four alternations
#
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6zj
for rep in 1 2 3 4; do
for cfg in "q192:--mask-queue 192" "q176:--mask-queue 176" "q160:--mask-queue 160"; do
  name=${cfg%%:*}; fl=${cfg#*:}
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline $fl > gpurun_out/${T}_${name}_$rep.json 2> gpurun_out/${T}_${name}_$rep.err || { tail -5 gpurun_out/${T}_${name}_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['config'].get('mask_schedule'))" gpurun_out/${T}_${name}_$rep.json $name
done
done
