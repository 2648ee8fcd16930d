# round 5q: configs[2] kernel trace (per-dispatch durations of the B = 1 chain)
set -o pipefail
mkdir -p gpurun_out
T=r5q
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex "k_" --output-format csv -d /tmp/pc -o c3 -- python3 bench.py --consecutive 32 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err || exit 1
find /tmp/pc -name "*kernel_trace.csv" -exec cp {} gpurun_out/${T}_c3_kernel_trace.csv \;
ls -la gpurun_out/${T}_c3_kernel_trace.csv
