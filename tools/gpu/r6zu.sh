# round 6zu: SQ issue / stall counters of the final build's serial bench (every kernel), two
# separate --pmc passes of <= 8 SQ counters each, then the per-wave table (tools/pmc_sq.py)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6zu
RX="--kernel-include-regex k_"
BS="python -u bench.py --serial --steps 3 --warmup 1 --no-cpu-baseline --distinct 32"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F64 $RX --output-format csv -d /tmp/q1 -o q -- $BS > gpurun_out/${T}_p1.log 2>&1 && echo P1_OK && \
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS $RX --output-format csv -d /tmp/q2 -o q -- $BS > gpurun_out/${T}_p2.log 2>&1 && echo P2_OK && \
python tools/pmc_sq.py $(find /tmp/q1 -name "*counter_collection.csv" | head -1) $(find /tmp/q2 -name "*counter_collection.csv" | head -1) --out gpurun_out/${T}_sq.json --note "final round-6 library, bench.py --serial" > gpurun_out/${T}_sq_table.txt && echo TABLE_OK && cat gpurun_out/${T}_sq_table.txt
