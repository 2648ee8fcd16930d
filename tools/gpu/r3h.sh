# round 3h: fix-up folded into k_select (per-frame lists), row tables prefetched in k_bin_curv:
# feature/edge/config tests, kernel-only feature chain times, latency line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3h_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 200 python -u tools/bench_features.py --reps 10 --chain > gpurun_out/r3h_feat.log 2>&1 && echo FEAT_OK && \
timeout -k 10 200 python -u bench.py --latency --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r3h_lat.json 2> gpurun_out/r3h_lat.err && echo LAT_OK
