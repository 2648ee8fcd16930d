# round 6w: pick_1m as a K1 walk + a bounded list walk (new default) vs one walk (ps0):
# registration tests on the default build, the table alone per build (same output hash), stamps
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6w
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_registration.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
for rep in 1 2; do
for v in def ps0; do
  if [ $v = def ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python3 -u tools/bench_table.py > gpurun_out/${T}_${v}_$rep.log 2>&1 || { tail gpurun_out/${T}_${v}_$rep.log; exit 1; }
  echo $v $(tail -1 gpurun_out/${T}_${v}_$rep.log)
done
done
SSF_LIB=$L/libssf_frontend_diag.so timeout -k 10 200 python3 -u tools/diag_table_phases.py 256 > gpurun_out/${T}_phases.log 2>&1 && cat gpurun_out/${T}_phases.log
