# round 3z: k-means++ prefetch depth 4 vs 2 (diag stamps)
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_kpp4.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r3z_kpp4.log 2>&1 && echo K4_OK && \
SSF_LIB=$L/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r3z_kpp2.log 2>&1 && echo K2_OK
