# round 6f: mask schedule in the full pipeline (longest-first by the previous launch on the same
# stream, frame queues), alternating, 60 steps; mask schedule parity test first
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6f
timeout -k 10 300 python -u -m pytest tests/test_gpu_mask.py -x -q --timeout 120 --timeout-method thread -k "schedule or golden" > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || exit 1
B="python3 -u bench.py --steps 60 --warmup 5 --no-cpu-baseline --kernel-pass 0"
for rep in 1 2; do
for v in base prev q192 q128p q192p; do
  case $v in base) X="";; prev) X="--mask-order prev";; q192) X="--mask-queue 192";; q128p) X="--mask-queue 128 --mask-order prev";; q192p) X="--mask-queue 192 --mask-order prev";; esac
  timeout -k 10 300 $B $X > gpurun_out/${T}_${v}_$rep.json 2> gpurun_out/${T}_${v}_$rep.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', round(d['value']), round(d['ms_per_step'],3))"
done
done
