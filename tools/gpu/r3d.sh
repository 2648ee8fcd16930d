# round 3d: streaming k_curv + lane-per-row k_select; tests, probe, latency, bench, consecutive
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3d_pytest.log 2>&1 && echo PYTEST_OK && \
for n in frontend cp2; do f=libssf_frontend_$n.so; [ $n = frontend ] && f=libssf_frontend.so; SSF_LIB=$L/$f timeout -k 10 200 python -u tools/bench_features.py --tag $n --reps 10 >> gpurun_out/r3d_probe.log 2>&1 || exit 1; done && echo PROBE_OK && \
timeout -k 10 200 python -u bench.py --latency --steps 30 --warmup 3 --no-cpu-baseline --mask-split 16 > gpurun_out/r3d_lat.json 2>/dev/null && echo LAT_OK && \
timeout -k 10 400 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r3d_bench.json 2> gpurun_out/r3d_bench.err && echo BENCH_OK && \
timeout -k 10 300 python -u bench.py --consecutive 32 --batch 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3d_consec.json 2> gpurun_out/r3d_consec.err && echo CONSEC_OK && \
timeout -k 10 300 python -u bench.py --mask-before-features --batch 32 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3d_c3.json 2> gpurun_out/r3d_c3.err && echo C3_OK
