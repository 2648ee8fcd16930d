# round 6zg: k_solve phase stamps -- ss1: compaction / first evaluation / iterations; ss2: the GN
# iterations split into the 6x6 solve + pose update and the evaluation (cycles per pair)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6zg
L=$PWD/ssf-slam_amd/ssf/_lib
for v in ss1 ss2 ss1 ss2; do
  SSF_LIB=$L/libssf_frontend_$v.so timeout -k 10 200 python3 -u tools/bench_features.py --chain --reps 4 --distinct 32 --stamps --tag $v >> gpurun_out/${T}_stamps.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/${T}_stamps.log
