# round 5bi: the default pipeline's ring depth 3 / 4 / 6, alternating (60 steps)
set -o pipefail
mkdir -p gpurun_out
T=r5bi
for rep in 1 2; do
for r in 4 3 6; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 60 --ring-depth $r > gpurun_out/${T}_${r}_$rep.json 2> gpurun_out/${T}_${r}_$rep.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${r}_$rep.json').read().strip().splitlines()[-1]);print('ring $r', round(d['value']), round(d['ms_per_step'],3), d['allocator_timed_region']['num_device_alloc'])"
done
done
