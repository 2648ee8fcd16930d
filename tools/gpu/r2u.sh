set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_edges.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2u_edges.log 2>&1
rc=$?; echo EDGES_RC=$rc
[ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r2u_pytest.log 2>&1
rc=$?; echo PYTEST_RC=$rc
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u tools/bench_features.py --tag edges_build --reps 5 --chain > gpurun_out/r2u_feat.log 2>&1 && echo FEAT_OK
