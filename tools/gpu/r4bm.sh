# round 4bm: the GPU suite at HEAD (incl. the outermost-window-column test of k_feat_wave_reg)
set -o pipefail
mkdir -p gpurun_out
T=r4bm
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo PYTEST_OK || { tail -40 gpurun_out/${T}_pytest_gpu.log; exit 1; }
