# round 4d: SQ / TA counter passes on the serial bench (every kernel alone on one stream):
# instructions per wave, issue and stall shares -- k_mask_pose's bound and the
# feature kernels' instruction mix (item 3)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CMD="python3 $R/bench.py --serial --steps 3 --warmup 1 --kernel-pass 0 --no-cpu-baseline"
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS" \
         "SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA" \
         "SQ_WAVES SQ_BUSY_CYCLES TA_BUSY_avr GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/r4d_sq$i -o p -- $CMD > $R/gpurun_out/r4d_sq$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok"
done
cd $R && python3 tools/pmc_sq.py $(ls gpurun_out/r4d_sq*/p_counter_collection.csv gpurun_out/r4d_sq*/*/p_counter_collection.csv 2>/dev/null) --out gpurun_out/r4d_sq.json --note "bench.py --serial --steps 3 --warmup 1, B=256 x 120k, HEAD build" > gpurun_out/r4d_sq_table.txt 2>&1; echo table rc=$?
