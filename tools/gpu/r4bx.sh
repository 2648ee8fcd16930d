# round 4bx: k_feat_wave_reg with the regularity margins folded into per-lane bounds (8 % fewer VALU) against the previous build (prev)
# (parity of the feature / config / edge / node / registration tests, alternating kernel-only times)
set -o pipefail
mkdir -p gpurun_out
T=r4bx
L=$GRAFT_REPO_ROOT/ssf-slam_amd/ssf/_lib
timeout -k 10 500 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_nodes.py tests/test_gpu_registration.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
for i in 1 2 3; do
  for v in default prev; do
    if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
    SSF_LIB=$lib timeout -k 10 120 python -u tools/bench_features.py --reps 5 --tag $v > gpurun_out/${T}_${v}_$i.json 2>&1 || exit 1
  done
done
echo FEAT_OK
