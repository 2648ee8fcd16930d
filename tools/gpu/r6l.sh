# round 6l: k_solve phase stamps (-DSSF_SOLVE_STAMPS) with and without the association-side
# compaction: compaction / first evaluation / iterations, cycles per pair
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6l
L=$PWD/ssf-slam_amd/ssf/_lib
for v in sstamp sstamp0 sstamp sstamp0; do
  SSF_LIB=$L/libssf_frontend_$v.so timeout -k 10 200 python3 -u tools/bench_features.py --chain --reps 4 --distinct 32 --stamps --tag $v >> gpurun_out/${T}_stamps.log 2>&1 || exit 1
done
echo STAMPS_OK
