# round 3am: the strip-image ABI checks test, then the profile set (r3ak)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_registration.py -x -q --timeout 120 --timeout-method thread -k "strip" > gpurun_out/r3am_pytest.log 2>&1 && echo PYTEST_OK && \
bash tools/gpu/r3ak.sh
