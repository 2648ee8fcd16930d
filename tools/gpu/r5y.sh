# round 5y: ssf_register_chain (configs[2] boundary pair + one chain call per step): tests, c3 lines
set -o pipefail
mkdir -p gpurun_out
T=r5y
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 500 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py tests/test_gpu_nodes.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
timeout -k 10 300 python3 bench.py --consecutive 32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_c3.json').read().strip().splitlines()[-1]);print('c3 chain', d['value'], d['ms_per_step'])"
timeout -k 10 300 python3 bench.py --consecutive 32 --steps 10 --warmup 3 --no-cpu-baseline --no-chain-api > gpurun_out/${T}_c3_pairwise.json 2> gpurun_out/${T}_c3_pairwise.err || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_c3_pairwise.json').read().strip().splitlines()[-1]);print('c3 pairwise', d['value'], d['ms_per_step'])"
timeout -k 10 300 python3 bench.py --consecutive 32 --steps 10 --warmup 3 --no-cpu-baseline --timeline > gpurun_out/${T}_c3_tl.json 2> gpurun_out/${T}_c3_tl.err || exit 1
tail -4 gpurun_out/${T}_c3_tl.err
