set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2d_feattest.log 2>&1 && echo TESTS_OK
