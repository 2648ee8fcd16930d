# round 4l: the point loads issued ahead of k_feat_chunk's set-up barrier (default) vs HEAD~ (prev)
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4l_pytest.log 2>&1 && echo PYTEST_OK || exit 1
for i in 1 2; do
  for v in default prev; do
    if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
    SSF_LIB=$lib timeout -k 10 120 python -u tools/bench_features.py --reps 5 --tag $v > gpurun_out/r4l_${v}_$i.json 2>&1 || exit 1
  done
done
echo ALL_OK
