# round 5n: k_solve LM state in registers (every thread) vs lane-0 step (lm0)
# builds (bench_features --chain, default layout), alternating
set -o pipefail
mkdir -p gpurun_out
T=r5n
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_nodes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || exit 1
for rep in 1 2; do
for v in both lm0; do
  if [ $v = both ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 tools/bench_features.py --reps 6 --chain > gpurun_out/${T}_${v}_$rep.json 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', d['kernel_ms']['k_solve'])"
done
done
# configs[2] as written: where the 4.8 ms step goes (per-step stage events)
timeout -k 10 300 python3 bench.py --consecutive 32 --steps 10 --warmup 3 --timeline > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err || exit 1
tail -4 gpurun_out/${T}_c3.err; python3 -c "import json;d=json.loads(open('gpurun_out/${T}_c3.json').read().strip().splitlines()[-1]);print('c3', d['value'], d['ms_per_step'])"
