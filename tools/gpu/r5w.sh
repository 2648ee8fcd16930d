# round 5w: SQ counters of k_associate_strips in the configs[2] chain (diag_chain_assoc, no deferral)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r5w
export SSF_LIB=$R/ssf-slam_amd/ssf/_lib/libssf_frontend_nodefer.so
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM" \
         "SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d /tmp/${T}_$i -o p -- python3 $R/tools/diag_chain_assoc.py 10 > $R/gpurun_out/${T}_sq$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 $R/tools/pmc_sq.py $(find /tmp/${T}_1 /tmp/${T}_2 /tmp/${T}_3 -name "p_counter_collection.csv") --out $R/gpurun_out/${T}_sq.json --note "tools/diag_chain_assoc.py 10: configs[2] chain, one pair per launch" > $R/gpurun_out/${T}_sq_table.txt 2>&1 && echo SQ_OK
cat $R/gpurun_out/${T}_sq_table.txt
