# round 5z: configs[2] as written at 30 timed steps (the round-4 line's length) + kernel trace
set -o pipefail
mkdir -p gpurun_out
T=r5z
timeout -k 10 300 python3 bench.py --consecutive 32 --steps 30 --warmup 3 > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_c3.json').read().strip().splitlines()[-1]);print('c3', d['value'], d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex "k_" --output-format csv -d /tmp/pc -o c3 -- python3 bench.py --consecutive 32 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c3tr.json 2> gpurun_out/${T}_c3tr.err || exit 1
find /tmp/pc -name "*kernel_trace.csv" -exec cp {} gpurun_out/${T}_c3_kernel_trace.csv \;
