set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BS="python -u bench.py --serial --steps 3 --warmup 1 --no-cpu-baseline --distinct 32"
RX="--kernel-include-regex k_"
timeout -k 10 300 rocprofv3 --list-avail > /tmp/avail.txt 2>&1; grep -i "F64\|FETCH_SIZE\|WRITE_SIZE" /tmp/avail.txt | head -40 > gpurun_out/r2h_avail_f64.txt; echo avail
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE $RX --output-format csv -d /tmp/pf -o f -- $BS > gpurun_out/r2h_pmc_fetch.log 2>&1 && echo FETCH_OK && \
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE $RX --output-format csv -d /tmp/pw -o w -- $BS > gpurun_out/r2h_pmc_write.log 2>&1 && echo WRITE_OK && \
python tools/pmc_traffic.py $(find /tmp/pf -name "*counter_collection.csv" | head -1) $(find /tmp/pw -name "*counter_collection.csv" | head -1) --bench-log gpurun_out/r2h_pmc_fetch.log --out gpurun_out/r2h_traffic.json > /dev/null && echo TRAFFIC_OK && \
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 $RX --output-format csv -d /tmp/pd -o d -- $BS > gpurun_out/r2h_pmc_f64.log 2>&1 && echo F64_OK && \
python tools/pmc_f64.py $(find /tmp/pd -name "*counter_collection.csv" | head -1) --bench-log gpurun_out/r2h_pmc_f64.log --out gpurun_out/r2h_f64.json > /dev/null && echo F64JSON_OK
ls -la /tmp/pf /tmp/pd 2>&1 | head; du -sh gpurun_out
