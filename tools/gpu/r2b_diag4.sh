set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_diag.so timeout -k 10 300 python -u tools/diag_mask_frames.py gpurun_out/mf_h0.npz 256 0 > gpurun_out/mf4.log 2>&1 && \
SSF_LIB=$L/libssf_frontend_diag.so timeout -k 10 300 python -u tools/diag_mask_frames.py gpurun_out/mf_h2.npz 256 2 >> gpurun_out/mf4.log 2>&1 && \
SSF_LIB=$L/libssf_frontend_diag.so timeout -k 10 300 python -u tools/diag_mask_frames.py gpurun_out/mf_h3.npz 256 3 >> gpurun_out/mf4.log 2>&1
