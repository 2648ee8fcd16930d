# round 5ai: PMC traffic (FETCH / WRITE) of the final build on the carla layout, then its line
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r05fin
RX="--kernel-include-regex k_"
BS="python -u bench.py --layout carla --serial --steps 3 --warmup 1 --no-cpu-baseline --distinct 32"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE $RX --output-format csv -d /tmp/pf -o f -- $BS > gpurun_out/${T}_carla_pmc_fetch.log 2>&1 && echo FETCH_OK && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE $RX --output-format csv -d /tmp/pw -o w -- $BS > gpurun_out/${T}_carla_pmc_write.log 2>&1 && echo WRITE_OK && \
python tools/pmc_traffic.py $(find /tmp/pf -name "*counter_collection.csv" | head -1) $(find /tmp/pw -name "*counter_collection.csv" | head -1) --bench-log gpurun_out/${T}_carla_pmc_fetch.log --out gpurun_out/${T}_carla_traffic.json > /dev/null && echo TRAFFIC_OK && \
cp gpurun_out/${T}_carla_traffic.json profiles/ && \
timeout -k 10 600 python -u bench.py --layout carla --steps 60 --no-cpu-baseline > gpurun_out/${T}_carla_line.json 2> gpurun_out/${T}_carla_line.err && echo LINE_OK
