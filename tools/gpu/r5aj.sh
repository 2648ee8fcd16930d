# round 5aj: the per-frame status test + the mask tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mask.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5aj_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/r5aj_pytest.log; exit 1; }
