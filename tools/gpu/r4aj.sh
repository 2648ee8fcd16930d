# round 4aj: the general kernel after k_feat_chunk_reg as k_feat_chunk_flagged (16 flags per work-group)
# (select derives positions, the regular kernel writes no u16 index): parity, times, PMC, bench
set -o pipefail
mkdir -p gpurun_out
T=r4aj
R=$PWD
L=$R/ssf-slam_amd/ssf/_lib
timeout -k 10 500 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_nodes.py tests/test_gpu_registration.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
for i in 1 2; do
  for v in default; do
    if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
    SSF_LIB=$lib timeout -k 10 120 python -u tools/bench_features.py --reps 5 --tag $v > gpurun_out/${T}_${v}_$i.json 2>&1 || exit 1
  done
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_def.json 2> gpurun_out/${T}_def.err && echo DEF && \
timeout -k 10 200 python -u bench.py --latency --no-cpu-baseline > gpurun_out/${T}_lat.json 2> gpurun_out/${T}_lat.err && echo LAT
