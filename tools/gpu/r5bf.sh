# round 5bf: per-wave deferral of EMPTY-region queries only (no candidate after the level)
# R = 2 or 4 (the 256-pair launch), vs no deferral; exactness on d4r2
set -o pipefail
mkdir -p gpurun_out
T=r5bf
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_e4r2.so timeout -k 10 500 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
for rep in 1 2; do
for v in both e4r2 e8r4 e16r4; do
  if [ $v = both ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 tools/bench_features.py --reps 6 --chain > gpurun_out/${T}_${v}_$rep.json 2>&1 || exit 1
  SSF_LIB=$lib timeout -k 10 300 python3 tools/bench_features.py --reps 6 --chain --layout carla > gpurun_out/${T}_${v}_c$rep.json 2>&1 || exit 1
  python3 -c "import json;a=json.loads(open('gpurun_out/${T}_${v}_$rep.json').read().strip().splitlines()[-1]);b=json.loads(open('gpurun_out/${T}_${v}_c$rep.json').read().strip().splitlines()[-1]);print('$v', a['kernel_ms']['k_associate_strips'], b['kernel_ms']['k_associate_strips'])"
done
done
