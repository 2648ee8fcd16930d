# round 5o: k_solve LM-in-registers A/B on the ceres_lm solver; configs[2] kernel stats (B = 1 chain)
set -o pipefail
mkdir -p gpurun_out
T=r5o
L=$PWD/ssf-slam_amd/ssf/_lib
for rep in 1 2; do
for v in both lm0; do
  if [ $v = both ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python3 tools/bench_features.py --reps 6 --chain --solver ceres_lm > gpurun_out/${T}_${v}_$rep.json 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', d['kernel_ms']['k_solve'])"
done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c3prof -o c3 -- python3 bench.py --consecutive 32 --steps 5 --warmup 2 > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err || exit 1
find gpurun_out/${T}_c3prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_c3_kernel_stats.csv \;
head -25 gpurun_out/${T}_c3_kernel_stats.csv | cut -d, -f1-8
