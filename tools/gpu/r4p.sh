# round 4p: where configs[2] (one sequence, 32 chained pairs per step) spends its time
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r4p
NB="--no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pk -o k -- python3 -u bench.py --consecutive 32 --steps 10 --warmup 2 $NB > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err && echo PROF_OK && \
cp $(find /tmp/pk -name "*kernel_stats.csv" | head -1) gpurun_out/${T}_c3_kernel_stats.csv && \
SSF_LIB=libssf_frontend_legacy.so timeout -k 10 300 python -u bench.py --consecutive 32 --steps 10 --warmup 2 $NB > gpurun_out/${T}_c3_legacy.json 2> gpurun_out/${T}_c3_legacy.err && echo LEG_OK
