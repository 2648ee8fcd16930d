# round 3ae: M-step wave form inlined vs called (diag stamps)
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_mi.so timeout -k 10 200 python -u tools/diag_mask_phases.py 1 > gpurun_out/r3ae_mi_b1.log 2>&1 && echo MI1_OK && \
SSF_LIB=$L/libssf_frontend_mi.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r3ae_mi_b256.log 2>&1 && echo MI256_OK
