set -o pipefail
mkdir -p gpurun_out
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_table_phases.py 256 > gpurun_out/tphase.log 2>&1
