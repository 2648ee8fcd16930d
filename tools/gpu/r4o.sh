# round 4o: PMC traffic of the product instantiations only (the kernel pass's debug launches are
# excluded by tools/pmc_traffic.py) -- FETCH / WRITE passes of the serial bench
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r4o
RX="--kernel-include-regex k_"
BS="python -u bench.py --serial --steps 3 --warmup 1 --no-cpu-baseline --distinct 32"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE $RX --output-format csv -d /tmp/pf -o f -- $BS > gpurun_out/${T}_pmc_fetch.log 2>&1 && echo FETCH_OK && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE $RX --output-format csv -d /tmp/pw -o w -- $BS > gpurun_out/${T}_pmc_write.log 2>&1 && echo WRITE_OK && \
cp $(find /tmp/pf -name "*counter_collection.csv" | head -1) gpurun_out/${T}_fetch.csv && cp $(find /tmp/pw -name "*counter_collection.csv" | head -1) gpurun_out/${T}_write.csv && \
python tools/pmc_traffic.py gpurun_out/${T}_fetch.csv gpurun_out/${T}_write.csv --bench-log gpurun_out/${T}_pmc_fetch.log --out gpurun_out/${T}_traffic.json > /dev/null && echo TRAFFIC_OK
