set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_registration.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2d_gntest.log 2>&1 && echo TESTS_OK
