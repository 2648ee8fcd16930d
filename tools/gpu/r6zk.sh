# round 6zk: Lloyd tunables on the round-6 data -- full passes before skipping (fp3 / fp5, default
# 4), record loads in flight (rd4 / rd12, default 8), back to a full pass above n / REFULL
# relabels (rf3 / rf6, default 4): mask alone, three streams, queue 192, alternating
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6zk
L=$PWD/ssf-slam_amd/ssf/_lib
for rep in 1 2; do
for v in def fp3 fp5 rd4 rd12 rf3 rf6; do
  if [ $v = def ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python3 -u tools/bench_mask_overlap.py --batch 256 --streams 3 --launches 24 --queue 192 > gpurun_out/${T}_mask_${v}_$rep.log 2>&1 || exit 1
  echo mask $v $(grep -o '"frames_per_s": [0-9.]*' gpurun_out/${T}_mask_${v}_$rep.log)
done
done
