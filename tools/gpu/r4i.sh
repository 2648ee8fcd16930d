# round 4i: k_feat_select with the staged transposition and LDS selections; why the sequences()
# path (configs[2]/[3]) is slower than the default bench per frame
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_configs.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4i_pytest.log 2>&1 && echo PYTEST_OK || exit 1
for i in 1 2; do
  for v in default zn0 exid legacy; do
    if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
    SSF_LIB=$lib timeout -k 10 120 python -u tools/bench_features.py --reps 5 --tag $v > gpurun_out/r4i_${v}_$i.json 2>&1 || exit 1
  done
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/r4i_default_bench.json 2> gpurun_out/r4i_default_bench.err || exit 1
timeout -k 10 300 python -u bench.py --sequences-total 256 --consecutive 1 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/r4i_seq256x1.json 2> gpurun_out/r4i_seq256x1.err || exit 1
timeout -k 10 300 python -u bench.py --sequences-total 256 --consecutive 1 --steps 20 --warmup 2 --kabsch-warm-start --no-cpu-baseline > gpurun_out/r4i_seq256x1_kws.json 2> gpurun_out/r4i_seq256x1_kws.err || exit 1
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 7 --warmup 1 --kabsch-warm-start --no-cpu-baseline > gpurun_out/r4i_c4_kws.json 2> gpurun_out/r4i_c4_kws.err || exit 1
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 7 --warmup 1 --kabsch-warm-start --mask-streams 2 --no-cpu-baseline > gpurun_out/r4i_c4_kws_ms2.json 2> gpurun_out/r4i_c4_kws_ms2.err || exit 1
echo ALL_OK
# SQ counters of the feature kernels alone (bench_features: features only, 5 reps)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/r4i_sq$i -o p -- python3 $R/tools/bench_features.py --reps 3 > $R/gpurun_out/r4i_sq$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
cd $R && python3 tools/pmc_sq.py $(find gpurun_out/r4i_sq1 gpurun_out/r4i_sq2 -name "p_counter_collection.csv") --out gpurun_out/r4i_sq.json --note "tools/bench_features.py --reps 3, B=256 x 120k" > gpurun_out/r4i_sq_table.txt 2>&1 && echo SQ_OK
cd $R
timeout -k 10 300 python -u bench.py --consecutive 32 --steps 10 --warmup 2 --kabsch-warm-start --mask-split 2 --no-cpu-baseline > gpurun_out/r4i_c3_kws_g2.json 2> gpurun_out/r4i_c3_kws_g2.err || exit 1
timeout -k 10 300 python -u bench.py --consecutive 32 --steps 10 --warmup 2 --kabsch-warm-start --mask-split 4 --no-cpu-baseline > gpurun_out/r4i_c3_kws_g4.json 2> gpurun_out/r4i_c3_kws_g4.err || exit 1
timeout -k 10 300 python -u bench.py --consecutive 32 --steps 10 --warmup 2 --kabsch-warm-start --no-cpu-baseline > gpurun_out/r4i_c3_kws_auto.json 2> gpurun_out/r4i_c3_kws_auto.err || exit 1
echo C3_OK
