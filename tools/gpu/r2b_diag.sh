set -o pipefail
mkdir -p gpurun_out
SSF_LIB=ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 300 python -u tools/diag_mask_frames.py gpurun_out/mask_frames.npz 256 > gpurun_out/mask_frames.log 2>&1
