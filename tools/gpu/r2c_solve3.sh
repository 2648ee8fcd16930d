set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
for n in frontend st256 st256s4 st256s1 st512s4 frontend st256 st256s4; do f=libssf_frontend_$n.so; [ $n = frontend ] && f=libssf_frontend.so; SSF_LIB=$L/$f timeout -k 10 200 python -u tools/bench_features.py --chain --reps 10 --tag $n --dump /tmp/p_$n.npz >> gpurun_out/r2c_solve3.log 2>&1 || exit 1; done && echo TIMING_OK
for n in st256 st256s4 st256s1 st512s4; do python -c "
import numpy as np
a=np.load('/tmp/p_frontend.npz'); b=np.load('/tmp/p_$n.npz')
d=np.abs(a['pose']-b['pose']); print('$n pose max |diff| vs default:', d.max())
" >> gpurun_out/r2c_solve3.log 2>&1; done; echo CMP_OK
