# round 5aq: plane-table pick walks over 0.5-m strips (five per 1-m region) vs 1-m strips (three):
# parity (registration + configs tests) and timing of the table and the association it images
set -o pipefail
mkdir -p gpurun_out
T=r5aq
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 500 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py tests/test_gpu_nodes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
for rep in 1 2; do
for v in both pickw1; do
  if [ $v = both ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 tools/bench_features.py --reps 6 --chain > gpurun_out/${T}_${v}_$rep.json 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$rep.json').read().strip().splitlines()[-1]);k=d['kernel_ms'];print('$v', k['k_plane_table_sorted'], k['k_associate_strips'])"
  SSF_LIB=$lib timeout -k 10 300 python3 tools/bench_features.py --reps 6 --chain --layout carla > gpurun_out/${T}_${v}_c$rep.json 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_c$rep.json').read().strip().splitlines()[-1]);k=d['kernel_ms'];print('$v carla', k['k_plane_table_sorted'], k['k_associate_strips'])"
done
done
