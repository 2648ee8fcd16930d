# round 4ac: k_feat_chunk_reg with the stencil's halo columns loaded from global memory (no LDS
# staging, no barriers) at 5 / 6 waves per SIMD vs the LDS-staged default
set -o pipefail
mkdir -p gpurun_out
T=r4ac
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_g5.so timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_g5.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest_g5.log; exit 1; }
for i in 1 2; do
  for v in default g5 g6; do
    if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
    SSF_LIB=$lib timeout -k 10 120 python -u tools/bench_features.py --reps 5 --tag $v > gpurun_out/${T}_${v}_$i.json 2>&1 || exit 1
  done
done
echo ALL_OK
