# round 5p: configs[2] kernel stats (B = 1 chain: per-pair association / solve latency)
set -o pipefail
mkdir -p gpurun_out
T=r5p
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pc -o c3 -- python3 bench.py --consecutive 32 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err || exit 1
find /tmp/pc -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_c3_kernel_stats.csv \;
head -25 gpurun_out/${T}_c3_kernel_stats.csv | cut -d, -f1-8
