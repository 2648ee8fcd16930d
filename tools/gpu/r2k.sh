set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r2k_gpu_tests.log 2>&1 && echo TESTS_OK && \
for v in old default; do
  L=ssf-slam_amd/ssf/_lib/libssf_frontend_$v.so; [ $v = default ] && L=ssf-slam_amd/ssf/_lib/libssf_frontend.so
  SSF_LIB=$PWD/$L timeout -k 10 120 python -u tools/bench_features.py --tag $v --reps 5 --chain >> gpurun_out/r2k_feat.log 2>&1 || exit 1
done && echo FEAT_OK
