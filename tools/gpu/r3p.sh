# round 3p: configs[1] latency with up to 64 mask parts per frame (split64 build) vs 32
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_split64.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mask.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3p_pytest.log 2>&1 && echo PYTEST_OK && \
for g in 32 48 64; do SSF_LIB=$L/libssf_frontend_split64.so timeout -k 10 200 python -u bench.py --latency --steps 40 --warmup 5 --no-cpu-baseline --mask-split $g > gpurun_out/r3p_lat_g$g.json 2>/dev/null || exit 1; done && echo LAT_OK && \
timeout -k 10 200 python -u bench.py --latency --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r3p_lat_default.json 2>/dev/null && echo LATD_OK
