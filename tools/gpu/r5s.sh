# round 5s: configs[2] chain: association work-group stamps (staging / queries / clock)
set -o pipefail
mkdir -p gpurun_out
T=r5s
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_sstamp.so timeout -k 10 300 python3 tools/diag_chain_assoc.py 12 > gpurun_out/${T}_stamps.log 2>&1 || exit 1
cat gpurun_out/${T}_stamps.log
