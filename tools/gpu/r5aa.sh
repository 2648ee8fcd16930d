# round 5aa: mask Infinity-Cache experiment: phase stamps per EM / Lloyd pass at
# B = 256 (G = 1, 737 MB of pos+flow in flight) vs B = 64 (G = 4, 184 MB: fits the 256 MiB MALL)
# vs B = 32 (G = 8, 92 MB), single stream, no chain
set -o pipefail
mkdir -p gpurun_out
T=r5aa
export SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so
for B in 256 64 32 256 64 32; do
  timeout -k 10 300 python3 tools/diag_mask_phases.py $B >> gpurun_out/${T}_phases.log 2>&1 || exit 1
done
cat gpurun_out/${T}_phases.log
