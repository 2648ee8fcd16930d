set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py tests/test_gpu_nodes.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2c_solve_tests.log 2>&1 && echo TESTS_OK || exit 1
for n in frontend qlibm st1024 st256 frontend qlibm; do f=libssf_frontend_$n.so; [ $n = frontend ] && f=libssf_frontend.so; SSF_LIB=$L/$f timeout -k 10 200 python -u tools/bench_features.py --chain --reps 10 --tag $n --dump /tmp/p_$n.npz >> gpurun_out/r2c_solve2.log 2>&1 || exit 1; done && echo TIMING_OK
SSF_LIB=$L/libssf_frontend_sstamp.so timeout -k 10 200 python -u tools/bench_features.py --chain --stamps --reps 5 --tag sstamp >> gpurun_out/r2c_solve2.log 2>&1 || exit 1
python -c "
import numpy as np
a=np.load('/tmp/p_frontend.npz'); b=np.load('/tmp/p_qlibm.npz')
print('normals/valid identical:', np.array_equal(a['normal'],b['normal']), np.array_equal(a['valid'],b['valid']))
d=np.abs(a['pose']-b['pose']); print('pose max |diff| taylor vs libm:', d.max(), 'identical entries', float((d==0).mean()))
" >> gpurun_out/r2c_solve2.log 2>&1; echo CMP_OK
