# round 5ax: rocprof kernel stats of configs[2] as written on the final build (the chain's
# per-pair association / solve and the step ring)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r05fin
timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_" --output-format csv -d /tmp/pc3 -o c -- python -u bench.py --consecutive 32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_c3_prof.log 2>&1 && echo C3PROF_OK && \
cp $(find /tmp/pc3 -name "*kernel_stats.csv" | head -1) gpurun_out/${T}_c3_kernel_stats.csv
