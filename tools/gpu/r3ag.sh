# round 3ag: plane-table phase stamps with the radix sort (diag build)
set -o pipefail
mkdir -p gpurun_out
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_table_phases.py 256 > gpurun_out/r3ag_table.log 2>&1 && echo T_OK
