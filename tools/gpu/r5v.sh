# round 5v: association work-group stamps: staging / lane pass / deferred pass
set -o pipefail
mkdir -p gpurun_out
T=r5v
L=$PWD/ssf-slam_amd/ssf/_lib
for v in sstamp0 sstamp sstamp8; do
SSF_LIB=$L/libssf_frontend_$v.so timeout -k 10 300 python3 tools/diag_chain_assoc.py 10 > gpurun_out/${T}_$v.log 2>&1 || exit 1
done
