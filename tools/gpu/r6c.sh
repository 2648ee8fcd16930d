# round 6c: k_solve specialised per solver mode (default) vs the shared kernel (spec0) vs
# specialised at 512 threads (s512): kernel-only chain times, alternating; registration parity
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6c
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || exit 1
for rep in 1 2 3; do
for v in def spec0 s512; do
  if [ $v = def ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python3 -u tools/bench_features.py --chain --reps 10 --distinct 32 --tag $v >> gpurun_out/${T}_feat.log 2>&1 || exit 1
done
done
echo AB_OK
