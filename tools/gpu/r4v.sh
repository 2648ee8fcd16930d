# round 4v: LDS counters of k_feat_chunk, whole kernel and the phase-cut timing variants
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=$R/ssf-slam_amd/ssf/_lib
P="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for v in default cut2 cut3 cut4; do
  if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d /tmp/r4v_$v -o p -- python3 $R/tools/bench_features.py --reps 3 > $R/gpurun_out/r4v_$v.log 2>&1 || { echo "pass $v failed"; exit 1; }
  python3 $R/tools/pmc_sq.py $(find /tmp/r4v_$v -name "p_counter_collection.csv") --out $R/gpurun_out/r4v_$v.json --note "$v" >> $R/gpurun_out/r4v_table.txt 2>&1 || exit 1
  echo "$v OK"
done
