set -o pipefail
mkdir -p gpurun_out
T=r5j
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python3 tools/bench_features.py --reps 8 --layout carla > gpurun_out/${T}_bf1.json 2>&1 && \
timeout -k 10 300 python3 tools/bench_features.py --reps 8 --layout carla > gpurun_out/${T}_bf2.json 2>&1 && echo BF_OK
