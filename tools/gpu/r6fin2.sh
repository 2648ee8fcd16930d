# round 6, final build part 2: the bench line of every config (profiles/r06fin_traffic.json,
# r06fin_carla_traffic.json and r06fin_f64.json from part 1, same library); the default line also
# at --warmup 60 and unstaggered (--stagger 0), and the one-GPU N = 2 gloo rehearsal (copy part 1's
# PMC JSONs from gpurun_out/ into profiles/ locally first: this call ships the local tree)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r06fin
run() { local name=$1; shift; timeout -k 10 600 python -u bench.py "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err && echo "${name}_OK" || { echo "${name}_FAIL"; tail -5 gpurun_out/${T}_$name.err; exit 1; }; }
run default_noflags
run w5 --steps 60 --warmup 5 --no-cpu-baseline
run w60 --steps 60 --warmup 60 --no-cpu-baseline
run w5s0 --steps 60 --warmup 5 --stagger 0 --no-cpu-baseline
run noqueue --steps 60 --warmup 5 --mask-queue 0 --no-cpu-baseline
run carla_line --layout carla --steps 60 --no-cpu-baseline
run c3 --consecutive 32 --steps 30 --warmup 3 --no-cpu-baseline
run c3kws --consecutive 32 --steps 30 --warmup 3 --kabsch-warm-start --no-cpu-baseline
run c4 --sequences-total 8 --consecutive 32 --steps 12 --warmup 2 --no-cpu-baseline
run c4kws --sequences-total 8 --consecutive 32 --steps 12 --warmup 2 --kabsch-warm-start --no-cpu-baseline
run c5 --n-az 4000 --steps 20 --no-cpu-baseline
run lat --latency --steps 40 --warmup 5 --no-cpu-baseline
run f64in --f64-inputs --steps 30 --no-cpu-baseline
run edges --edges --steps 30 --no-cpu-baseline
timeout -k 10 600 python -u bench.py --gpus 2 --rehearse-one-gpu --steps 20 --no-cpu-baseline --batch 128 > gpurun_out/${T}_n2_rehearsal.json 2> gpurun_out/${T}_n2_rehearsal.err && echo N2_OK
echo PART2_DONE
