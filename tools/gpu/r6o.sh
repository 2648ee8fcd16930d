# round 6o: Huber weights by refined v_rcp_f64 (hrcp) vs the f64 divide (default), GN-specialised solve: parity, kernel times
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6o
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py tests/test_gpu_nodes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
for rep in 1 2 3; do
for v in def hrcp; do
  if [ $v = def ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python3 -u tools/bench_features.py --chain --reps 10 --distinct 32 --tag $v >> gpurun_out/${T}_feat.log 2>&1 || exit 1
done
done
echo AB_OK
