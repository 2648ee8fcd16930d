# round 4br: chain stream priority (high, the default, vs normal), alternating, 30 steps
set -o pipefail
mkdir -p gpurun_out
T=r4br
B="python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline"
for i in 1 2 3; do
  timeout -k 10 200 $B > gpurun_out/${T}_prio_hi_$i.json 2>/dev/null && echo hi-$i || exit 1
  timeout -k 10 200 $B --feat-priority 0 > gpurun_out/${T}_prio_0_$i.json 2>/dev/null && echo p0-$i || exit 1
done
