# round 5ba: feature + registration + config tests with one output per thread per trip in k_feat_select
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_configs.py tests/test_gpu_nodes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5ba_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/r5ba_pytest.log; exit 1; }
