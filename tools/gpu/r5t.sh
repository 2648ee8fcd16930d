# round 5t: configs[2] chain: association stamps per work-group + strip-search counts
set -o pipefail
mkdir -p gpurun_out
T=r5t
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_sstamp.so timeout -k 10 300 python3 tools/diag_chain_assoc.py 12 > gpurun_out/${T}_stamps.log 2>&1 || exit 1
SSF_LIB=$L/libssf_frontend_acount.so timeout -k 10 300 python3 tools/diag_chain_assoc.py 12 > gpurun_out/${T}_count.log 2>&1 || exit 1
cat gpurun_out/${T}_stamps.log gpurun_out/${T}_count.log
