set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_xext.so timeout -k 10 400 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2d_xext_tests.log 2>&1 && echo TESTS_OK || exit 1
for n in frontend xext frontend xext; do f=libssf_frontend_$n.so; [ $n = frontend ] && f=libssf_frontend.so; echo "== $n" >> gpurun_out/r2d_xext.log; SSF_LIB=$L/$f timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --mask-before-features --batch 32 --dump-poses /tmp/x_$n.npy >> gpurun_out/r2d_xext.log 2>&1 || exit 1; SSF_LIB=$L/$f timeout -k 10 200 python -u tools/bench_features.py --chain --reps 10 --tag $n --dump /tmp/xf_$n.npz >> gpurun_out/r2d_xext.log 2>&1 || exit 1; done && echo AB_OK
python -c "
import numpy as np
a=np.load('/tmp/x_frontend.npy'); b=np.load('/tmp/x_xext.npy'); print('c3 poses identical:', np.array_equal(a.view(np.uint64), b.view(np.uint64)))
" >> gpurun_out/r2d_xext.log && python tools/cmp_npz.py /tmp/xf_frontend.npz /tmp/xf_xext.npz >> gpurun_out/r2d_xext.log && echo CMP_OK
