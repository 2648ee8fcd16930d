# round 3e: k_curv scalar prologue, k_select prefetch/batched emit, parallel mask exchange gather
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3e_pytest.log 2>&1 && echo PYTEST_OK && \
for n in frontend cp2; do f=libssf_frontend_$n.so; [ $n = frontend ] && f=libssf_frontend.so; SSF_LIB=$L/$f timeout -k 10 200 python -u tools/bench_features.py --tag $n --reps 10 >> gpurun_out/r3e_probe.log 2>&1 || exit 1; done && echo PROBE_OK && \
for g in 8 16 32; do timeout -k 10 200 python -u bench.py --latency --steps 30 --warmup 3 --no-cpu-baseline --mask-split $g > gpurun_out/r3e_lat_g$g.json 2>/dev/null || exit 1; done && echo LAT_OK && \
timeout -k 10 400 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r3e_bench.json 2> gpurun_out/r3e_bench.err && echo BENCH_OK && \
timeout -k 10 300 python -u bench.py --mask-before-features --batch 32 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3e_c3.json 2> gpurun_out/r3e_c3.err && echo C3_OK
