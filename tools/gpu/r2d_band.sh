set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
s=$(date +%s); timeout -k 10 500 python -u bench.py > gpurun_out/r2d_band_default.log 2>&1 && echo "DEFAULT_OK $(( $(date +%s) - s )) s" || exit 1
for k in 1 2 3; do timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2d_band_$k.log 2>&1 || exit 1; done && echo BAND_OK
