# round 5au: sequence-mode ring depth 5 vs 8 vs 12 (configs[2] / configs[3], Kabsch warm starts and chained)
set -o pipefail
mkdir -p gpurun_out
T=r5au
run() { local name=$1; shift; timeout -k 10 600 python -u bench.py "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { echo "${name}_FAIL"; tail -8 gpurun_out/${T}_$name.err; exit 1; }; python3 -c "import json;d=json.loads(open('gpurun_out/${T}_$name.json').read().strip().splitlines()[-1]);print('$name', round(d['value']), round(d['ms_per_step'],3), d['allocator_timed_region']['num_device_alloc'])"; }
for r in 5 8 12; do
run c3kws_$r --consecutive 32 --steps 30 --warmup 3 --kabsch-warm-start --no-cpu-baseline --seq-ring $r
run c4kws_$r --sequences-total 8 --consecutive 32 --steps 12 --warmup 2 --kabsch-warm-start --no-cpu-baseline --seq-ring $r
run c3_$r --consecutive 32 --steps 30 --warmup 3 --no-cpu-baseline --seq-ring $r
done
