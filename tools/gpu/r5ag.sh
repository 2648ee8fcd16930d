# round 5ag: is the no-flag line's ~8 % deficit a cold start? fresh box: default line first with
# warmup 5, then warmup 50, then warmup 5 again (GPU now warm), then the no-flag run with CPU legs
set -o pipefail
mkdir -p gpurun_out
T=r5ag
run() { local name=$1; shift; timeout -k 10 600 python -u bench.py "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { echo "${name}_FAIL"; exit 1; }; python3 -c "import json;d=json.loads(open('gpurun_out/${T}_$name.json').read().strip().splitlines()[-1]);print('$name', round(d['value']), round(d['ms_per_step'],3))"; }
run w5_cold --no-cpu-baseline --warmup 5
run w50 --no-cpu-baseline --warmup 50
run w5_warm --no-cpu-baseline --warmup 5
run noflags
run noflags_w50 --warmup 50
