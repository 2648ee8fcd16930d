# round 4t: persistent k_feat_chunk (resident grid, optional next-chunk prefetch) vs the r4m build
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_configs.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4t_pytest.log 2>&1 && echo PYTEST_OK || exit 1
for i in 1 2; do
  for v in default r4m nores pf5 pf4; do
    if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
    SSF_LIB=$lib timeout -k 10 120 python -u tools/bench_features.py --reps 5 --tag $v > gpurun_out/r4t_${v}_$i.json 2>&1 || exit 1
  done
done
echo ALL_OK
