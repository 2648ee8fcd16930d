# round 5ar: the group-cooperative association for big launches too (2 / 4 / 8 lanes per query,
# one work-group per pair, queries looped) vs the lane mode; registration tests on big4
set -o pipefail
mkdir -p gpurun_out
T=r5ar
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_big4.so timeout -k 10 500 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
for rep in 1 2; do
for v in both big2 big4 big8; do
  if [ $v = both ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 tools/bench_features.py --reps 6 --chain > gpurun_out/${T}_${v}_$rep.json 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$rep.json').read().strip().splitlines()[-1]);k=d['kernel_ms'];print('$v', k['k_associate_strips'])"
done
done
