# round 5ae: k_solve (256 pairs) phase stamps and SQ counter passes -- VERDICT r4 item 5's counter table
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r5ae
SSF_LIB=$R/ssf-slam_amd/ssf/_lib/libssf_frontend_sstamps.so timeout -k 10 300 python3 $R/tools/bench_features.py --reps 3 --chain --stamps > $R/gpurun_out/${T}_stamps.log 2>&1 || exit 1
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM" \
         "SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d /tmp/${T}_$i -o p -- python3 $R/tools/bench_features.py --reps 3 --chain > $R/gpurun_out/${T}_sq$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/${T}_sq$i.log; exit 1; }
done
python3 $R/tools/pmc_sq.py $(find /tmp/${T}_1 /tmp/${T}_2 /tmp/${T}_3 /tmp/${T}_4 -name "p_counter_collection.csv") --out $R/gpurun_out/${T}_sq.json --note "tools/bench_features.py --reps 3 --chain: 256 pairs per k_solve launch" > $R/gpurun_out/${T}_sq_table.txt 2>&1 && echo SQ_OK
grep k_solve $R/gpurun_out/${T}_sq_table.txt; tail -2 $R/gpurun_out/${T}_stamps.log
