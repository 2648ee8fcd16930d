set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
for v in diag diagd12 diagl3 diag; do
SSF_LIB=$L/libssf_frontend_$v.so timeout -k 10 300 python -u tools/diag_mask_frames.py gpurun_out/mf_$v.npz 256 >> gpurun_out/mf_deep.log 2>&1 || exit 1
python tools/diag_mask_summary.py gpurun_out/mf_$v.npz >> gpurun_out/mf_deep.log 2>&1
done
