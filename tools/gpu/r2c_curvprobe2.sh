set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2c_feat_tests.log 2>&1 && SSF_LIB=$L/libssf_frontend_bc2048.so timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py -x -q --timeout 120 --timeout-method thread >> gpurun_out/r2c_feat_tests.log 2>&1 && echo FEAT_OK || exit 1
for n in frontend cp1 cp3 cp3d6 cp2 bc2048 bc1024 frontend; do f=libssf_frontend_$n.so; [ $n = frontend ] && f=libssf_frontend.so; SSF_LIB=$L/$f timeout -k 10 200 python -u tools/bench_features.py --tag $n --reps 10 >> gpurun_out/r2c_curvprobe2.log 2>&1 || exit 1; done && echo PROBE_OK
