set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2s_pytest.log 2>&1 && echo PYTEST_OK && \
for lib in noseed frontend; do n=libssf_frontend_$lib.so; [ $lib = frontend ] && n=libssf_frontend.so; SSF_LIB=$L/$n timeout -k 10 200 python -u tools/bench_features.py --tag $lib --reps 5 --chain >> gpurun_out/r2s_ab.log 2>&1 || exit 1; done && echo AB_OK && \
for lib in noseed frontend; do n=libssf_frontend_$lib.so; [ $lib = frontend ] && n=libssf_frontend.so; SSF_LIB=$L/$n timeout -k 10 200 python -u tools/bench_features.py --tag ${lib}_c5 --n-az 4000 --reps 3 --chain >> gpurun_out/r2s_ab.log 2>&1 || exit 1; done && echo AB5_OK
