# round 4a: the float32 Kabsch tail (a19) -- mask tests on the device
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mask.py tests/test_abi.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4a_pytest.log 2>&1 && echo PYTEST_OK
