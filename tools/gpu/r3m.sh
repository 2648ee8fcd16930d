# round 3m: Lloyd candidate lists in a non-inlined skip-pass function: mask tests, A/B vs the
# previous kernel (bit-identical masks), phase stamps of both
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_mask.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3m_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 200 python -u tools/bench_mask.py --batch 256 --splits 1 --reps 3 --distinct 256 --dump /tmp/new256.npz > gpurun_out/r3m_mask256_new.log 2>&1 && echo M1_OK && \
SSF_LIB=$L/libssf_frontend_head.so timeout -k 10 200 python -u tools/bench_mask.py --batch 256 --splits 1 --reps 3 --distinct 256 --dump /tmp/head256.npz > gpurun_out/r3m_mask256_head.log 2>&1 && echo M2_OK && \
python tools/cmp_npz.py /tmp/new256.npz /tmp/head256.npz > gpurun_out/r3m_cmp256.log && echo CMP1_OK && \
timeout -k 10 200 python -u tools/bench_mask.py --batch 32 --splits 8 --reps 3 --dump /tmp/new32.npz > gpurun_out/r3m_mask32_new.log 2>&1 && echo M3_OK && \
SSF_LIB=$L/libssf_frontend_head.so timeout -k 10 200 python -u tools/bench_mask.py --batch 32 --splits 8 --reps 3 --dump /tmp/head32.npz > gpurun_out/r3m_mask32_head.log 2>&1 && echo M4_OK && \
python tools/cmp_npz.py /tmp/new32.npz /tmp/head32.npz > gpurun_out/r3m_cmp32.log && echo CMP2_OK && \
SSF_LIB=$L/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r3m_diag_new.log 2>&1 && echo D1_OK && \
SSF_LIB=$L/libssf_frontend_diaghead.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r3m_diag_head.log 2>&1 && echo D2_OK
