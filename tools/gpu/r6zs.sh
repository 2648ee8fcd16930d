# round 6zs: k-means++ prefetch depth (kd1 / kd4, default 2) and the Lloyd streamer depth (ld1 / ld3,
# default 2) on the final loops: mask alone, three streams, queue 192, alternating
#
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6zs
L=$PWD/ssf-slam_amd/ssf/_lib
for rep in 1 2; do
for v in def kd1 kd4 ld1 ld3; do
  if [ $v = def ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python3 -u tools/bench_mask_overlap.py --batch 256 --streams 3 --launches 24 --queue 192 > gpurun_out/${T}_mask_${v}_$rep.log 2>&1 || exit 1
  echo mask $v $(grep -o '"frames_per_s": [0-9.]*' gpurun_out/${T}_mask_${v}_$rep.log)
done
done
