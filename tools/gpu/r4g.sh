# round 4g: VERDICT r3 item 4 -- the E-step parameters as SGPR operands (-DSSF_EM_SGPR) against the
# per-pair LDS reads: mean frame stamp cycles (diagnostic builds), alternating, same box
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
for i in 1 2; do
  SSF_LIB=$L/libssf_frontend_diag.so timeout -k 10 120 python -u tools/diag_mask_phases.py 256 > gpurun_out/r4g_base_$i.log 2>&1 || exit 1
  SSF_LIB=$L/libssf_frontend_emsgpr_diag.so timeout -k 10 120 python -u tools/diag_mask_phases.py 256 > gpurun_out/r4g_sgpr_$i.log 2>&1 || exit 1
done
echo AB_OK
