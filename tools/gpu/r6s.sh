# round 6s: k_feat_wave_run (carla layout) A/B -- the interior test as one ballot (b1), the
# register step as the buffer load's SGPR offset (soff), 4 registers in flight (pf4) vs the
# default (3 in flight, three ballots), kernel-only times, alternating
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6s
L=$PWD/ssf-slam_amd/ssf/_lib
for rep in 1 2 3; do
for v in def b1 soff pf4; do
  if [ $v = def ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python3 -u tools/bench_features.py --layout carla --reps 10 --distinct 32 --tag $v >> gpurun_out/${T}_feat.log 2>&1 || exit 1
done
done
echo AB_OK
