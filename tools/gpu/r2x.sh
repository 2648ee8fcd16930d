set -o pipefail
mkdir -p gpurun_out
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_acount.so timeout -k 10 200 python -u tools/diag_assoc_count.py 64 > gpurun_out/r2x_count.log 2>&1 && echo COUNT_OK
