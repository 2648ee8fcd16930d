# round 4an: k_feat_chunk_reg without per-load integer multiplies (uniform column offsets)
set -o pipefail
mkdir -p gpurun_out
T=r4an
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/bench_features.py --reps 5 --tag default > gpurun_out/${T}_default_$i.json 2>&1 || exit 1
done
echo ALL_OK
