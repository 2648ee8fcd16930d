# round 3g: fused binning + curvature (k_bin_curv, k_curv_fixup, flag-byte k_select): GPU suite,
# serial kernel pass, default bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3g_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python -u bench.py --serial --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3g_serial.json 2> gpurun_out/r3g_serial.err && echo SERIAL_OK && \
timeout -k 10 400 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r3g_bench.json 2> gpurun_out/r3g_bench.err && echo BENCH_OK && \
timeout -k 10 200 python -u bench.py --latency --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r3g_lat.json 2> gpurun_out/r3g_lat.err && echo LAT_OK && \
timeout -k 10 300 python -u bench.py --consecutive 32 --batch 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3g_consec.json 2> gpurun_out/r3g_consec.err && echo CONSEC_OK
