set -o pipefail
mkdir -p gpurun_out
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r3w2_phases_b256.log 2>&1 && echo PH256_OK
