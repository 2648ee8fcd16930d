# round 3x: Lloyd skip pass with 12 record loads in flight per lane (diag stamps) vs 8
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r3x_rd8.log 2>&1 && echo RD8_OK && \
SSF_LIB=$L/libssf_frontend_rd12.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r3x_rd12.log 2>&1 && echo RD12_OK
