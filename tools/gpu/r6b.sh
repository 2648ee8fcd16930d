# round 6b: the steady-car generator (cars wrap round the ego) + staggered sequence starts:
# per-step serial costs along the sequences, and the default line at warmup 5 / 60, stagger 200 / 0
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6b
timeout -k 10 300 python -u tools/diag_mask_window.py gpurun_out/${T}_window.json 150 > gpurun_out/${T}_window.log 2>&1 && echo WIN_OK && \
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_w5.json 2> gpurun_out/${T}_w5.err && echo W5_OK && \
timeout -k 10 300 python -u bench.py --steps 40 --warmup 60 --no-cpu-baseline > gpurun_out/${T}_w60.json 2> gpurun_out/${T}_w60.err && echo W60_OK && \
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --stagger 0 --no-cpu-baseline > gpurun_out/${T}_w5s0.json 2> gpurun_out/${T}_w5s0.err && echo W5S0_OK && \
timeout -k 10 300 python -u bench.py --steps 40 --warmup 60 --stagger 0 --no-cpu-baseline > gpurun_out/${T}_w60s0.json 2> gpurun_out/${T}_w60s0.err && echo W60S0_OK
