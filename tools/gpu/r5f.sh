# round 5f: k_feat_wave_run with the lean steady state (interior uniform registers, masks by v_writelane)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r5f
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python3 tools/bench_features.py --reps 5 --layout carla > gpurun_out/${T}_bf_carla.json 2>&1 && echo BF_OK && \
timeout -k 10 300 python3 tools/bench_features.py --reps 5 > gpurun_out/${T}_bf_default.json 2>&1 && echo BF2_OK || exit 1
cd /tmp
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d /tmp/${T}_$i -o p -- python3 $R/tools/bench_features.py --reps 3 --layout carla > $R/gpurun_out/${T}_sq$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 $R/tools/pmc_sq.py $(find /tmp/${T}_1 /tmp/${T}_2 -name "p_counter_collection.csv") --out $R/gpurun_out/${T}_sq.json --note "bench_features --reps 3 --layout carla" > $R/gpurun_out/${T}_sq_table.txt 2>&1 && echo SQ_OK
