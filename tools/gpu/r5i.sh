# round 5i: the carla layout keeps the off-road ground (rm_road removes the road only): tests + line
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r5i
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py -x -q --timeout 120 --timeout-method thread -k "carla or run_kernel" > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 400 python -u bench.py --layout carla --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_carla.json 2> gpurun_out/${T}_carla.err && echo CARLA_OK && \
timeout -k 10 300 python3 tools/bench_features.py --reps 5 --layout carla --chain > gpurun_out/${T}_bf_carla.json 2>&1 && echo BF_OK
