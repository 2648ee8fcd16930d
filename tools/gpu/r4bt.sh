# round 4bt: HEAD as the driver runs it: the GPU suite, smoke, the no-flag bench line
set -o pipefail
mkdir -p gpurun_out
T=r4bt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_default_noflags.json 2> gpurun_out/${T}_default_noflags.err && echo NOFLAGS
