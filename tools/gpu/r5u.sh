# round 5u: association far queries deferred to a wave each: exactness (registration tests),
# chain diagnostics (stamps, counts) and the configs[2] line, deferred vs not
set -o pipefail
mkdir -p gpurun_out
T=r5u
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || exit 1
SSF_LIB=$L/libssf_frontend_acount0.so timeout -k 10 300 python3 tools/diag_chain_assoc.py 12 > gpurun_out/${T}_count0.log 2>&1 || exit 1
SSF_LIB=$L/libssf_frontend_acount.so timeout -k 10 300 python3 tools/diag_chain_assoc.py 12 > gpurun_out/${T}_count.log 2>&1 || exit 1
SSF_LIB=$L/libssf_frontend_sstamp.so timeout -k 10 300 python3 tools/diag_chain_assoc.py 12 > gpurun_out/${T}_stamps.log 2>&1 || exit 1
for v in both nodefer; do
  if [ $v = both ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 bench.py --consecutive 32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_c3_$v.json 2> gpurun_out/${T}_c3_$v.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_c3_$v.json').read().strip().splitlines()[-1]);print('c3 $v', d['value'], d['ms_per_step'])"
  SSF_LIB=$lib timeout -k 10 300 python3 tools/bench_features.py --reps 6 --chain > gpurun_out/${T}_feat_$v.json 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_feat_$v.json').read().strip().splitlines()[-1]);print('256 $v', {k: v for k, v in d['kernel_ms'].items() if 'assoc' in k})"
done
