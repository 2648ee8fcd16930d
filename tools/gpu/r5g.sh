# round 5g: k_feat_wave_run, fewer VALU in the steady state
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r5g
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python3 tools/bench_features.py --reps 5 --layout carla > gpurun_out/${T}_bf_carla.json 2>&1 && echo BF_OK && \
timeout -k 10 300 python3 tools/bench_features.py --reps 5 --layout carla > gpurun_out/${T}_bf_carla2.json 2>&1 && echo BF2_OK
