# round 5am: k_solve with J^T W J accumulated in packed f32 (hf32) -- parity tests on that library
# and timing vs f64 (GN and LM)
set -o pipefail
mkdir -p gpurun_out
T=r5am
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_hf32.so timeout -k 10 500 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py tests/test_gpu_nodes.py tests/test_gpu_edges.py -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; tail -15 gpurun_out/${T}_pytest.log
for s in gn ceres_lm; do
for rep in 1 2; do
for v in both hf32; do
  if [ $v = both ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 tools/bench_features.py --reps 6 --chain --solver $s > gpurun_out/${T}_${v}_$s$rep.json 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$s$rep.json').read().strip().splitlines()[-1]);print('$v $s', d['kernel_ms']['k_solve'])"
done
done
done
