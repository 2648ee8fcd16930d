# round 6zv: k_mask_pose phase shares (stamp build) of the final loops at frames 0 and 100
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$PWD/ssf-slam_amd/ssf/_lib
for k in 0 100; do
  SSF_LIB=$L/libssf_frontend_diag.so timeout -k 10 200 python3 -u tools/diag_mask_phases.py 256 $k > gpurun_out/r6zv_phases_$k.log 2>&1 || exit 1
  cat gpurun_out/r6zv_phases_$k.log
done
