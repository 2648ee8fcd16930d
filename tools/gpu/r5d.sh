# round 5d: k_feat_wave_run registers in flight (SSF_FEAT_RUN_PF 2 / 4 / 6 / 8), A/B on the carla layout
set -o pipefail
mkdir -p gpurun_out
T=r5d
L=ssf-slam_amd/ssf/_lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py -x -q --timeout 120 --timeout-method thread -k "carla or run_kernel" > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK && \
for v in pf4 pf2 pf6 pf8 pf4; do
  if [ $v = pf4 ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --layout carla --steps 10 --warmup 2 --no-cpu-baseline --distinct 32 > gpurun_out/${T}_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${T}_$v.json'));print('$v', d['kernels']['k_feat_wave_run']['ms'], d['kernels']['k_feat_wave_run'].get('frac'))"
done
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_default.json 2> gpurun_out/${T}_default.err && echo DEFAULT_OK && \
timeout -k 10 400 python -u bench.py --f64-inputs --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_f64in.json 2> gpurun_out/${T}_f64in.err && echo F64_OK
