# round 6h: mask frame-queue size sweep in the full pipeline (60 steps), and mask streams 2 / 4
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6h
B="python3 -u bench.py --steps 60 --warmup 5 --no-cpu-baseline --kernel-pass 0"
for rep in 1 2; do
for v in q96 q128 q160 q192 q224 q160s2 q192s4 q128s4; do
  case $v in q96) X="--mask-queue 96";; q128) X="--mask-queue 128";; q160) X="--mask-queue 160";; q192) X="--mask-queue 192";; q224) X="--mask-queue 224";;
             q160s2) X="--mask-queue 160 --mask-streams 2";; q192s4) X="--mask-queue 192 --mask-streams 4";; q128s4) X="--mask-queue 128 --mask-streams 4";; esac
  timeout -k 10 300 $B $X > gpurun_out/${T}_${v}_$rep.json 2> gpurun_out/${T}_${v}_$rep.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', round(d['value']), round(d['ms_per_step'],3))"
done
done
