# round 5al: k_solve with the Jacobian's factor 2 folded into the block sums: bit-identical poses
# (GN and LM, dumps compared as raw bits) and timing vs the per-correspondence factor (jscale0)
set -o pipefail
mkdir -p gpurun_out
T=r5al
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
for s in gn ceres_lm; do
for v in both jscale0; do
  if [ $v = both ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 tools/bench_features.py --reps 6 --chain --solver $s --dump gpurun_out/${T}_${v}_$s.npz > gpurun_out/${T}_${v}_$s.json 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$s.json').read().strip().splitlines()[-1]);print('$v $s', d['kernel_ms']['k_solve'])"
done
python3 tools/cmp_npz.py gpurun_out/${T}_both_$s.npz gpurun_out/${T}_jscale0_$s.npz
done
