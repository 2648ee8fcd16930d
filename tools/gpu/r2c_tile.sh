set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2c_tile_tests.log 2>&1 && echo TESTS_OK || exit 1
for n in frontend frontend; do SSF_LIB=$L/libssf_frontend.so timeout -k 10 200 python -u tools/bench_features.py --tag tile --reps 10 >> gpurun_out/r2c_tile.log 2>&1 || exit 1; done && echo PROBE_OK
