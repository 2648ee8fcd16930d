# round 5r: configs[2] chain: per-pair association time vs walk statistics
set -o pipefail
mkdir -p gpurun_out
T=r5r
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 300 python3 tools/diag_chain_assoc.py > gpurun_out/${T}_time.log 2>&1 || exit 1
SSF_LIB=$L/libssf_frontend_acount.so timeout -k 10 300 python3 tools/diag_chain_assoc.py > gpurun_out/${T}_count.log 2>&1 || exit 1
cat gpurun_out/${T}_time.log gpurun_out/${T}_count.log
