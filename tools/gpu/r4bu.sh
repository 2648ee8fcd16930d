# round 4bu: SQ counters of the final build's chain kernels (k_feat_wave_reg, select, plane table, association, solve) --
# bench_features --chain, three passes
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS" \
         "SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d /tmp/r4bu_$i -o p -- python3 $R/tools/bench_features.py --reps 3 --chain > $R/gpurun_out/r4bu_sq$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 $R/tools/pmc_sq.py $(find /tmp/r4bu_1 /tmp/r4bu_2 /tmp/r4bu_3 -name "p_counter_collection.csv") --out $R/gpurun_out/r4bu_sq.json --note "tools/bench_features.py --reps 3 --chain, B=256 x 120k" > $R/gpurun_out/r4bu_sq_table.txt 2>&1 && echo SQ_OK
