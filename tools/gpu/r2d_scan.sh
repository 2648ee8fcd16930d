set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2d_scan_tests.log 2>&1 && echo TESTS_OK || exit 1
timeout -k 10 200 python -u tools/bench_features.py --chain --reps 10 --tag scan > gpurun_out/r2d_scan.log 2>&1 && echo TIMING_OK || exit 1
SSF_LIB=$L/libssf_frontend_diag.so timeout -k 10 300 python -u tools/diag_mask_phases.py > gpurun_out/r2d_phases.log 2>&1 && echo PHASES_OK
