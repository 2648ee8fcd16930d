# round 3ad: M-step over the 64 lanes of wave 0 vs the two-lane form: bitwise A/B (B = 256, 1 part;
# B = 1, 32 parts; B = 33, automatic), mask tests, diag stamps, bench
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
for c in "256 1" "1 32" "33 0"; do set -- $c
SSF_LIB=$L/libssf_frontend_m2.so timeout -k 10 200 python -u tools/dump_mask.py $1 $2 gpurun_out/r3ad_m2_$1.npz > gpurun_out/r3ad_dump.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/dump_mask.py $1 $2 gpurun_out/r3ad_mw_$1.npz >> gpurun_out/r3ad_dump.log 2>&1 || exit 1
python tools/cmp_npz.py gpurun_out/r3ad_m2_$1.npz gpurun_out/r3ad_mw_$1.npz >> gpurun_out/r3ad_cmp.log && rm -f gpurun_out/r3ad_m2_$1.npz gpurun_out/r3ad_mw_$1.npz || exit 1
done
echo CMP_OK && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_mask.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3ad_pytest.log 2>&1 && echo PYTEST_OK && \
SSF_LIB=$L/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r3ad_phases_b256.log 2>&1 && echo PH256_OK && \
SSF_LIB=$L/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_mask_phases.py 1 > gpurun_out/r3ad_phases_b1.log 2>&1 && echo PH1_OK && \
timeout -k 10 300 python -u bench.py --latency --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r3ad_latency.log 2>&1 && echo LAT_OK && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3ad_bench.log 2>&1 && echo BENCH_OK
