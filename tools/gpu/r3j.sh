# round 3j: register-resident 5x3 QR (no scratch in the plane table), exchange fences on by
# default: GPU suite, feature/table chain times, PMC traffic of the table
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RX="--kernel-include-regex k_"
BS="python -u bench.py --serial --steps 3 --warmup 1 --no-cpu-baseline --distinct 32"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3j_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 200 python -u tools/bench_features.py --reps 10 --chain > gpurun_out/r3j_feat.log 2>&1 && echo FEAT_OK && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE $RX --output-format csv -d /tmp/pf -o f -- $BS > gpurun_out/r3j_pmc_fetch.log 2>&1 && echo FETCH_OK && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE $RX --output-format csv -d /tmp/pw -o w -- $BS > gpurun_out/r3j_pmc_write.log 2>&1 && echo WRITE_OK && \
python tools/pmc_traffic.py $(find /tmp/pf -name "*counter_collection.csv" | head -1) $(find /tmp/pw -name "*counter_collection.csv" | head -1) --bench-log gpurun_out/r3j_pmc_fetch.log --out gpurun_out/r3j_traffic.json > /dev/null && echo TRAFFIC_OK
