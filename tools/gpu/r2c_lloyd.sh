set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
for n in diag dlf2 dlf3 drf2 drf8; do echo "== $n" >> gpurun_out/r2c_lloyd.log; SSF_LIB=$L/libssf_frontend_$n.so timeout -k 10 200 python -u tools/diag_mask_frames.py /tmp/m_$n.npz 256 >> gpurun_out/r2c_lloyd.log 2>&1 || exit 1; done && echo DIAG_OK
for n in dlf2 dlf3 drf2 drf8; do python -c "import numpy as np,sys; a=np.load('/tmp/m_diag.npz')['out'][:, :26]; b=np.load('/tmp/m_$n.npz')['out'][:, :26]; print('$n results identical (cols 0-25, bitwise):', np.array_equal(a.view(np.uint32) if a.dtype==np.float32 else a.view(np.uint64), b.view(np.uint32) if b.dtype==np.float32 else b.view(np.uint64)))" >> gpurun_out/r2c_lloyd.log 2>&1; done; echo CMP_DONE
for n in frontend lf3 rf8 frontend lf3 rf8; do f=libssf_frontend_$n.so; [ $n = frontend ] && f=libssf_frontend.so; echo "== $n" >> gpurun_out/r2c_lloyd_bench.log; SSF_LIB=$L/$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/r2c_lloyd_bench.log 2>&1 || exit 1; done && echo BENCH_OK
