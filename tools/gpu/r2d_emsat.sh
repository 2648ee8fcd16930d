set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
for n in diag dsat746 dsat40; do echo "== $n" >> gpurun_out/r2d_emsat.log; SSF_LIB=$L/libssf_frontend_$n.so timeout -k 10 300 python -u tools/diag_mask_phases.py >> gpurun_out/r2d_emsat.log 2>&1 || exit 1; SSF_LIB=$L/libssf_frontend_$n.so timeout -k 10 200 python -u tools/diag_mask_frames.py /tmp/e_$n.npz 256 >> gpurun_out/r2d_emsat.log 2>&1 || exit 1; done && echo DIAG_OK
for n in dsat746 dsat40; do python -c "
import numpy as np
a=np.load('/tmp/e_diag.npz')['out'][:, :26]; b=np.load('/tmp/e_$n.npz')['out'][:, :26]
v=lambda x: x.view(np.uint64) if x.dtype==np.float64 else x.view(np.uint32)
print('$n identical cols 0-25:', np.array_equal(v(a), v(b)), 'iters equal:', np.array_equal(a[:,19:21], b[:,19:21]), 'max |dt|:', float(np.abs(a[:,0:3]-b[:,0:3]).max()))
" >> gpurun_out/r2d_emsat.log 2>&1; done; echo CMP_DONE
