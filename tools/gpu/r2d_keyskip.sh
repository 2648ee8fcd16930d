set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2d_keyskip_tests.log 2>&1 && echo TESTS_OK || exit 1
for n in frontend ks0 frontend ks0; do f=libssf_frontend_$n.so; [ $n = frontend ] && f=libssf_frontend.so; SSF_LIB=$L/$f timeout -k 10 200 python -u tools/bench_features.py --chain --reps 10 --tag $n --dump /tmp/k_$n.npz >> gpurun_out/r2d_keyskip.log 2>&1 || exit 1; done && echo TIMING_OK
for n in frontend ks0; do f=libssf_frontend_$n.so; [ $n = frontend ] && f=libssf_frontend.so; SSF_LIB=$L/$f timeout -k 10 200 python -u tools/bench_features.py --chain --reps 5 --n-az 4000 --tag c5_$n --dump /tmp/k5_$n.npz >> gpurun_out/r2d_keyskip.log 2>&1 || exit 1; done && echo C5_OK
python tools/cmp_npz.py /tmp/k_frontend.npz /tmp/k_ks0.npz >> gpurun_out/r2d_keyskip.log && python tools/cmp_npz.py /tmp/k5_frontend.npz /tmp/k5_ks0.npz >> gpurun_out/r2d_keyskip.log && echo CMP_OK
