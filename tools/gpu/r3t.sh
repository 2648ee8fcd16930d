# round 3t: plane-table phase stamps (diag build) after the register-resident QR
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_table_phases.py 256 > gpurun_out/r3t_table.log 2>&1 && echo T_OK
