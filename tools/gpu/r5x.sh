# round 5x: group-cooperative association for few-pair launches (coop16 default, coop8, coop0 = lane mode)
set -o pipefail
mkdir -p gpurun_out
T=r5x
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py tests/test_gpu_nodes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || exit 1
SSF_LIB=$L/libssf_frontend_sstamp.so timeout -k 10 300 python3 tools/diag_chain_assoc.py 10 > gpurun_out/${T}_stamps.log 2>&1 || exit 1
for v in both coop8 coop0; do
  if [ $v = both ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 tools/diag_chain_assoc.py 12 > gpurun_out/${T}_chain_$v.log 2>&1 || exit 1
  SSF_LIB=$lib timeout -k 10 300 python3 bench.py --consecutive 32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_c3_$v.json 2> gpurun_out/${T}_c3_$v.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_c3_$v.json').read().strip().splitlines()[-1]);print('c3 $v', d['value'], d['ms_per_step'])"
done
