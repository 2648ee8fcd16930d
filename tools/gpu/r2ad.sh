set -o pipefail
mkdir -p gpurun_out
for r in 6 8 12; do SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_dr$r.so timeout -k 10 200 python -u tools/diag_table_phases.py 256 > gpurun_out/r2ad_table_dr$r.log 2>&1 || exit 1; done && echo TABLE_OK
