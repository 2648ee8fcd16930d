# round 6zt: k_feat_wave_run occupancy bound (rw4 / rw6, default 8 waves per SIMD) and registers
# in flight (rpf2, default 3) on carla-layout frames: the kernel alone (tools/bench_features.py
# --layout carla, ms per 256-frame launch), alternating
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6zt
L=$PWD/ssf-slam_amd/ssf/_lib
for rep in 1 2 3; do
for v in def rw4 rw6 rpf2; do
  if [ $v = def ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python3 -u tools/bench_features.py --layout carla --reps 8 --distinct 32 --tag $v > gpurun_out/${T}_${v}_$rep.log 2>&1 || { tail gpurun_out/${T}_${v}_$rep.log; exit 1; }
  echo $v $(grep -o '"k_feat_wave_run": [0-9.]*' gpurun_out/${T}_${v}_$rep.log)
done
done
