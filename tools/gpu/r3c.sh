# round 3c: greedy on SGPRs (readfirstlane wave index) -- probes, features tests, latency splits,
# bench with the bounded ego heading
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_edges.py tests/test_gpu_mask.py tests/test_gpu_registration.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c_pytest.log 2>&1 && echo PYTEST_OK && \
for n in frontend cp1 cp2; do f=libssf_frontend_$n.so; [ $n = frontend ] && f=libssf_frontend.so; SSF_LIB=$L/$f timeout -k 10 200 python -u tools/bench_features.py --tag $n --reps 10 >> gpurun_out/r3c_probe.log 2>&1 || exit 1; done && echo PROBE_OK && \
for g in 8 16 32; do timeout -k 10 200 python -u bench.py --latency --steps 30 --warmup 3 --no-cpu-baseline --mask-split $g > gpurun_out/r3c_lat_g$g.json 2>/dev/null || exit 1; done && echo LAT_OK && \
timeout -k 10 400 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r3c_bench.json 2> gpurun_out/r3c_bench.err && echo BENCH_OK && \
timeout -k 10 300 python -u bench.py --consecutive 32 --batch 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3c_consec.json 2> gpurun_out/r3c_consec.err && echo CONSEC_OK
