# round 4f: single-read feature stage -- parity tests, then kernel times of the variants
# (default = scalar stencil at 5 waves/SIMD; pk5 / pk4 = packed-f32 stencil at 5 / 4; sc4 =
# scalar at 4; legacy = the round-3 four-kernel stage), alternating, same box
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 500 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_registration.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4f_pytest.log 2>&1 && echo PYTEST_OK || exit 1
for i in 1 2; do
  for v in default pk5 pk4 sc4 legacy; do
    if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
    SSF_LIB=$lib timeout -k 10 120 python -u tools/bench_features.py --reps 5 --tag $v > gpurun_out/r4f_${v}_$i.json 2>&1 || exit 1
  done
done
echo BENCH_OK
