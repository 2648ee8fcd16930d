# round 4w: k_feat_chunk without LDS write bank conflicts (swizzled own-tile slots and flags,
# one pad float per row run of the tile): parity first, then times and LDS counters vs r4m
set -o pipefail
mkdir -p gpurun_out
R=$PWD
L=$R/ssf-slam_amd/ssf/_lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_nodes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4w_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/r4w_pytest.log; exit 1; }
for i in 1 2; do
  for v in default r4m; do
    if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
    SSF_LIB=$lib timeout -k 10 120 python -u tools/bench_features.py --reps 5 --tag $v > gpurun_out/r4w_${v}_$i.json 2>&1 || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
P="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d /tmp/r4w_lds -o p -- python3 $R/tools/bench_features.py --reps 3 > $R/gpurun_out/r4w_lds.log 2>&1 && \
python3 $R/tools/pmc_sq.py $(find /tmp/r4w_lds -name "p_counter_collection.csv") --out $R/gpurun_out/r4w_lds.json --note "swizzled k_feat_chunk" > $R/gpurun_out/r4w_lds.txt 2>&1 && echo ALL_OK
