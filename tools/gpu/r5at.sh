# round 5at: the sequence modes with the step ring: allocator growth and the lines (configs[2] /
# configs[3], chained and Kabsch warm starts, and B = 2 sequences: the per-pair path)
set -o pipefail
mkdir -p gpurun_out
T=r5at
run() { local name=$1; shift; timeout -k 10 600 python -u bench.py "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { echo "${name}_FAIL"; tail -8 gpurun_out/${T}_$name.err; exit 1; }; python3 -c "import json;d=json.loads(open('gpurun_out/${T}_$name.json').read().strip().splitlines()[-1]);print('$name', round(d['value']), round(d['ms_per_step'],3), d['allocator_timed_region'], d.get('poses_finite'), round(d.get('final_t_norm',0),3))"; }
run c3 --consecutive 32 --steps 30 --warmup 3 --no-cpu-baseline
run c3kws --consecutive 32 --steps 30 --warmup 3 --kabsch-warm-start --no-cpu-baseline
run c4 --sequences-total 8 --consecutive 32 --steps 12 --warmup 2 --no-cpu-baseline
run c4kws --sequences-total 8 --consecutive 32 --steps 12 --warmup 2 --kabsch-warm-start --no-cpu-baseline
run c3b2 --consecutive 8 --batch 2 --steps 10 --warmup 2 --no-cpu-baseline
