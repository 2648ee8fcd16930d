# round 6m: plane table pick keys carrying the ring code (two other-ring keys instead of six) and
# k_solve's LDS prefetch: registration / configs / node parity, then kernel times vs pf0 (no
# LDS prefetch) and cmp0 (round-5 table and association, no compaction), alternating
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6m
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py tests/test_gpu_nodes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
for rep in 1 2 3; do
for v in def pf0 cmp0; do
  if [ $v = def ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python3 -u tools/bench_features.py --chain --reps 10 --distinct 32 --tag $v >> gpurun_out/${T}_feat.log 2>&1 || exit 1
done
done
echo AB_OK
