# round 3ai: Lloyd block summaries -- bitwise A/B against the per-point skip pass, mask tests,
# diag stamps of both, overlapped bench of both
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
for c in "256 1" "1 32" "33 0"; do set -- $c
SSF_LIB=$L/libssf_frontend_nb.so timeout -k 10 200 python -u tools/dump_mask.py $1 $2 gpurun_out/r3ai_a_$1.npz > gpurun_out/r3ai_dump.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/dump_mask.py $1 $2 gpurun_out/r3ai_b_$1.npz >> gpurun_out/r3ai_dump.log 2>&1 || exit 1
python tools/cmp_npz.py gpurun_out/r3ai_a_$1.npz gpurun_out/r3ai_b_$1.npz >> gpurun_out/r3ai_cmp.log && rm -f gpurun_out/r3ai_a_$1.npz gpurun_out/r3ai_b_$1.npz || exit 1
done
echo CMP_OK && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_mask.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3ai_pytest.log 2>&1 && echo PYTEST_OK && \
SSF_LIB=$L/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r3ai_blk_b256.log 2>&1 && echo PHB_OK && \
SSF_LIB=$L/libssf_frontend_nbdiag.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r3ai_pt_b256.log 2>&1 && echo PHP_OK && \
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --kernel-pass 1 > gpurun_out/r3ai_blk_$r.log 2>&1 || exit 1
SSF_LIB=$L/libssf_frontend_nb.so timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --kernel-pass 1 > gpurun_out/r3ai_pt_$r.log 2>&1 || exit 1
done && echo AB_OK
