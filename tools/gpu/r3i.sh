# round 3i: PMC traffic of every chain kernel (fused features, staged plane table), rocprof
# kernel-trace stats of the serial bench, the configs[2] B=32 line, mask split sweep for the
# configs[1] latency line, exchange fences A/B on latency and configs[2]
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$PWD/ssf-slam_amd/ssf/_lib
RX="--kernel-include-regex k_"
BS="python -u bench.py --serial --steps 3 --warmup 1 --no-cpu-baseline --distinct 32"
timeout -k 10 300 rocprofv3 --kernel-trace --stats $RX --output-format csv -d /tmp/ps -o s -- python -u bench.py --serial --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3i_serial_bench.log 2>&1 && echo SERIAL_OK && \
cp $(find /tmp/ps -name "*kernel_stats.csv" | head -1) gpurun_out/r3i_serial_kernel_stats.csv && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE $RX --output-format csv -d /tmp/pf -o f -- $BS > gpurun_out/r3i_pmc_fetch.log 2>&1 && echo FETCH_OK && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE $RX --output-format csv -d /tmp/pw -o w -- $BS > gpurun_out/r3i_pmc_write.log 2>&1 && echo WRITE_OK && \
python tools/pmc_traffic.py $(find /tmp/pf -name "*counter_collection.csv" | head -1) $(find /tmp/pw -name "*counter_collection.csv" | head -1) --bench-log gpurun_out/r3i_pmc_fetch.log --out gpurun_out/r3i_traffic.json > /dev/null && echo TRAFFIC_OK && \
timeout -k 10 300 python -u bench.py --mask-before-features --batch 32 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3i_c3.json 2> gpurun_out/r3i_c3.err && echo C3_OK && \
for g in 8 16 32; do timeout -k 10 200 python -u bench.py --latency --steps 40 --warmup 5 --no-cpu-baseline --mask-split $g > gpurun_out/r3i_lat_g$g.json 2>/dev/null || exit 1; done && echo LAT_OK && \
SSF_LIB=$L/libssf_frontend_fences.so timeout -k 10 200 python -u bench.py --latency --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r3i_lat_fences.json 2>/dev/null && echo LATF_OK && \
timeout -k 10 300 python -u bench.py --consecutive 32 --batch 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3i_consec.json 2>/dev/null && echo CONSEC_OK && \
SSF_LIB=$L/libssf_frontend_fences.so timeout -k 10 300 python -u bench.py --consecutive 32 --batch 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3i_consec_fences.json 2>/dev/null && echo CONSECF_OK
