# round 5ad: plane table phase stamps with the 4-lane deferred groups (diag build); tests
set -o pipefail
mkdir -p gpurun_out
T=r5ad
timeout -k 10 400 python -u -m pytest tests/test_gpu_registration.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 300 python3 tools/diag_table_phases.py 256 > gpurun_out/${T}_phases.log 2>&1 || exit 1
cat gpurun_out/${T}_phases.log
