# round 4c: the counter names this rocprofv3 offers on gfx950 (for the SQ/TA passes)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r4c_counters.txt 2>&1; echo rc=$?
