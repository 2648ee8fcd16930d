# round 5, final build part 2: the bench line of every config (profiles/r05fin_traffic.json and
# r05fin_f64.json from part 1, same library)
set -o pipefail
mkdir -p gpurun_out
T=r05fin
run() { local name=$1; shift; timeout -k 10 600 python -u bench.py "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err && echo "${name}_OK" || { echo "${name}_FAIL"; tail -5 gpurun_out/${T}_$name.err; exit 1; }; }
run default_noflags
run carla --layout carla --steps 30 --no-cpu-baseline
run carla_line --layout carla --steps 60 --no-cpu-baseline
run c3 --consecutive 32 --steps 30 --warmup 3 --no-cpu-baseline
run c3kws --consecutive 32 --steps 30 --warmup 3 --kabsch-warm-start --no-cpu-baseline
run c4 --sequences-total 8 --consecutive 32 --steps 12 --warmup 2 --no-cpu-baseline
run c4kws --sequences-total 8 --consecutive 32 --steps 12 --warmup 2 --kabsch-warm-start --no-cpu-baseline
run c5 --n-az 4000 --steps 20 --no-cpu-baseline
run lat --latency --steps 40 --warmup 5 --no-cpu-baseline
run f64in --f64-inputs --steps 30 --no-cpu-baseline
run edges --edges --steps 30 --no-cpu-baseline
echo PART2_DONE
