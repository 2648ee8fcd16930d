# round 3l: k_mask_pose phase stamps, candidate-list build vs the previous kernel (diag builds)
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r3l_diag_new.log 2>&1 && echo D1_OK && \
SSF_LIB=$L/libssf_frontend_diaghead.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r3l_diag_head.log 2>&1 && echo D2_OK
