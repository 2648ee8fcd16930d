# round 5e: SQ counters of k_feat_wave_run on the carla layout (bench_features --layout carla), three passes;
# plus the ring A/B of the f64-inputs line (the round-4 185 ms stall: allocator retries?)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r5e
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM" \
         "SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d /tmp/${T}_$i -o p -- python3 $R/tools/bench_features.py --reps 3 --layout carla > $R/gpurun_out/${T}_sq$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 $R/tools/pmc_sq.py $(find /tmp/${T}_1 /tmp/${T}_2 /tmp/${T}_3 -name "p_counter_collection.csv") --out $R/gpurun_out/${T}_sq.json --note "tools/bench_features.py --reps 3 --layout carla, B=256 x 120k" > $R/gpurun_out/${T}_sq_table.txt 2>&1 && echo SQ_OK
cd $R
timeout -k 10 400 python -u bench.py --f64-inputs --no-ring --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_f64in_noring.json 2> gpurun_out/${T}_f64in_noring.err && echo NORING_OK && \
timeout -k 10 400 python -u bench.py --f64-inputs --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_f64in_ring.json 2> gpurun_out/${T}_f64in_ring.err && echo RING_OK && \
timeout -k 10 300 python -u bench.py --no-ring --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_def_noring.json 2> gpurun_out/${T}_def_noring.err && echo NORING2_OK
