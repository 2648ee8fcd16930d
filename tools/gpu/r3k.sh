# round 3k: Lloyd candidate lists -- mask tests, A/B against the previous kernel (HEAD build,
# libssf_frontend_head.so) at B = 256 (G = 1) and B = 32 (G = 8), outputs compared bit for bit,
# then the default bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3k_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 200 python -u tools/bench_mask.py --batch 256 --splits 1 --reps 3 --distinct 256 --dump /tmp/new256.npz > gpurun_out/r3k_mask256_new.log 2>&1 && echo M1_OK && \
SSF_LIB=$L/libssf_frontend_head.so timeout -k 10 200 python -u tools/bench_mask.py --batch 256 --splits 1 --reps 3 --distinct 256 --dump /tmp/head256.npz > gpurun_out/r3k_mask256_head.log 2>&1 && echo M2_OK && \
python tools/cmp_npz.py /tmp/new256.npz /tmp/head256.npz > gpurun_out/r3k_cmp256.log && echo CMP1_OK && \
timeout -k 10 200 python -u tools/bench_mask.py --batch 32 --splits 8 --reps 3 --dump /tmp/new32.npz > gpurun_out/r3k_mask32_new.log 2>&1 && echo M3_OK && \
SSF_LIB=$L/libssf_frontend_head.so timeout -k 10 200 python -u tools/bench_mask.py --batch 32 --splits 8 --reps 3 --dump /tmp/head32.npz > gpurun_out/r3k_mask32_head.log 2>&1 && echo M4_OK && \
python tools/cmp_npz.py /tmp/new32.npz /tmp/head32.npz > gpurun_out/r3k_cmp32.log && echo CMP2_OK && \
timeout -k 10 400 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r3k_bench.json 2> gpurun_out/r3k_bench.err && echo BENCH_OK && \
timeout -k 10 200 python -u bench.py --latency --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r3k_lat.json 2> gpurun_out/r3k_lat.err && echo LAT_OK && \
timeout -k 10 300 python -u bench.py --consecutive 32 --batch 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3k_consec.json 2> gpurun_out/r3k_consec.err && echo CONSEC_OK && \
timeout -k 10 300 python -u bench.py --mask-before-features --batch 32 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3k_c3.json 2> gpurun_out/r3k_c3.err && echo C3_OK
