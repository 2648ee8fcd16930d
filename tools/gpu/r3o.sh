# round 3o: k_bin_curv with 4096-point chunks on 512-thread work-groups (sub2) vs 2048 / 256:
# feature tests on both, kernel-only chain times
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_sub2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3o_pytest_sub2.log 2>&1 && echo PYTEST2_OK && \
for n in frontend sub2 frontend sub2; do f=libssf_frontend_$n.so; [ $n = frontend ] && f=libssf_frontend.so; SSF_LIB=$L/$f timeout -k 10 200 python -u tools/bench_features.py --tag $n --reps 10 >> gpurun_out/r3o_feat.log 2>&1 || exit 1; done && echo FEAT_OK
