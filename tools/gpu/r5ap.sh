# round 5ap: feature tests with 3 registers in flight in k_feat_wave_run
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_features.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5ap_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/r5ap_pytest.log; exit 1; }
