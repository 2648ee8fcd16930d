# round 3s: k_bin_curv ranks with per-row LDS lane words instead of the 6-bit ballot match
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_edges.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3s_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 200 python -u tools/bench_features.py --reps 10 > gpurun_out/r3s_feat.log 2>&1 && \
timeout -k 10 200 python -u tools/bench_features.py --reps 10 >> gpurun_out/r3s_feat.log 2>&1 && echo FEAT_OK
