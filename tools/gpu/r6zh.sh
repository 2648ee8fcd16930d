# round 6zh: k_solve's first evaluation with every record of a thread requested at once (new:
# default build, SSF_SOLVE_LOADALL) vs one step ahead (la0): registration tests, the kernel alone
# (tools/bench_features.py --chain, k_solve ms per 256-pair launch), stamps of the new build
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6zh
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_registration.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
for rep in 1 2 3; do
for v in la0 new; do
  if [ $v = new ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python3 -u tools/bench_features.py --chain --reps 6 --distinct 32 --tag $v > gpurun_out/${T}_${v}_$rep.log 2>&1 || { tail gpurun_out/${T}_${v}_$rep.log; exit 1; }
  echo $v $(grep -o '"k_solve": [0-9.]*' gpurun_out/${T}_${v}_$rep.log) $(grep -o '"k_associate_strips": [0-9.]*' gpurun_out/${T}_${v}_$rep.log)
done
done
SSF_LIB=$L/libssf_frontend_lastamp.so timeout -k 10 200 python3 -u tools/bench_features.py --chain --reps 4 --distinct 32 --stamps --tag lastamp 2>&1 | grep solve_stamps
