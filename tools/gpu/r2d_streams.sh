set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do for ms in 2 3 4; do echo "== ms$ms" >> gpurun_out/r2d_streams.log; timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --mask-streams $ms --kernel-pass 0 >> gpurun_out/r2d_streams.log 2>&1 || exit 1; done; done && echo STREAMS_OK
