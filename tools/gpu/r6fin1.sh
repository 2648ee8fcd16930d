# round 6, final build part 1: every GPU test, smoke, and the profile set -- PMC traffic (FETCH /
# WRITE, separate passes) and the mask's f64 issue counters on the serial bench, rocprof kernel
# stats of the serial / overlapped default bench, the configs[1] latency run and the carla layout
# (serial + its PMC traffic); the PMC JSONs go to profiles/ here so that part 2's lines read them
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r06fin
RX="--kernel-include-regex k_"
BS="python -u bench.py --serial --steps 3 --warmup 1 --no-cpu-baseline --distinct 32"
BC="python -u bench.py --layout carla --serial --steps 3 --warmup 1 --no-cpu-baseline --distinct 32"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && echo SMOKE_OK && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE $RX --output-format csv -d /tmp/pf -o f -- $BS > gpurun_out/${T}_pmc_fetch.log 2>&1 && echo FETCH_OK && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE $RX --output-format csv -d /tmp/pw -o w -- $BS > gpurun_out/${T}_pmc_write.log 2>&1 && echo WRITE_OK && \
python tools/pmc_traffic.py $(find /tmp/pf -name "*counter_collection.csv" | head -1) $(find /tmp/pw -name "*counter_collection.csv" | head -1) --bench-log gpurun_out/${T}_pmc_fetch.log --out gpurun_out/${T}_traffic.json > /dev/null && echo TRAFFIC_OK && \
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 $RX --output-format csv -d /tmp/pd2 -o d -- $BS > gpurun_out/${T}_pmc_f64.log 2>&1 && echo F64_OK && \
python tools/pmc_f64.py $(find /tmp/pd2 -name "*counter_collection.csv" | head -1) --bench-log gpurun_out/${T}_pmc_f64.log --out gpurun_out/${T}_f64.json > /dev/null && echo F64JSON_OK && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE $RX --output-format csv -d /tmp/pcf -o f -- $BC > gpurun_out/${T}_carla_pmc_fetch.log 2>&1 && echo CFETCH_OK && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE $RX --output-format csv -d /tmp/pcw -o w -- $BC > gpurun_out/${T}_carla_pmc_write.log 2>&1 && echo CWRITE_OK && \
python tools/pmc_traffic.py $(find /tmp/pcf -name "*counter_collection.csv" | head -1) $(find /tmp/pcw -name "*counter_collection.csv" | head -1) --bench-log gpurun_out/${T}_carla_pmc_fetch.log --out gpurun_out/${T}_carla_traffic.json > /dev/null && echo CTRAFFIC_OK && \
cp gpurun_out/${T}_traffic.json gpurun_out/${T}_f64.json gpurun_out/${T}_carla_traffic.json profiles/ && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats $RX --output-format csv -d /tmp/ps -o s -- python -u bench.py --serial --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_serial_bench.log 2>&1 && echo SERIAL_OK && \
cp $(find /tmp/ps -name "*kernel_stats.csv" | head -1) gpurun_out/${T}_serial_kernel_stats.csv && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats $RX --output-format csv -d /tmp/pd -o d -- python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_default_bench.log 2>&1 && echo DEFAULT_OK && \
cp $(find /tmp/pd -name "*kernel_stats.csv" | head -1) gpurun_out/${T}_default_kernel_stats.csv && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats $RX --output-format csv -d /tmp/pl -o l -- python -u bench.py --latency --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_latency.log 2>&1 && echo LATENCY_OK && \
cp $(find /tmp/pl -name "*kernel_stats.csv" | head -1) gpurun_out/${T}_latency_kernel_stats.csv && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats $RX --output-format csv -d /tmp/pc -o c -- python -u bench.py --layout carla --serial --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_carla_serial.log 2>&1 && echo CARLA_SERIAL_OK && \
cp $(find /tmp/pc -name "*kernel_stats.csv" | head -1) gpurun_out/${T}_carla_serial_kernel_stats.csv && echo PART1_DONE
