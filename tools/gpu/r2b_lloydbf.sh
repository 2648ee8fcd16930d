set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_diag.so timeout -k 10 300 python -u tools/diag_mask_frames.py gpurun_out/mf_bf.npz 256 > gpurun_out/mf_bf.log 2>&1 && \
timeout -k 10 200 python -u tools/bench_mask.py --batch 256 --splits 1 --reps 3 --distinct 256 --dump gpurun_out/bf_cur.npz >> gpurun_out/mf_bf.log 2>&1
