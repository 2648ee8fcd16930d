# round 5bh: the whole GPU suite and smoke on HEAD (the round-end driver's two GPU steps)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5bh_pytest_gpu.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5bh_smoke.log 2>&1 && echo SMOKE_OK
