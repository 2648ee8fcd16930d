# round 6za: same-box pipeline A/B -- r06fin library (old), the current one (new), the current
# one with the round-6 register-prefetch EM (em1); default line at 60 steps, alternating
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6za
L=$PWD/ssf-slam_amd/ssf/_lib
for rep in 1 2 3; do
for v in old new em1; do
  if [ $v = new ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_${v}_$rep.json 2> gpurun_out/${T}_${v}_$rep.err || { tail -5 gpurun_out/${T}_${v}_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['roofline']['frac'])" gpurun_out/${T}_${v}_$rep.json $v
done
done
for v in old new; do
  if [ $v = new ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python3 -u tools/bench_mask_overlap.py --batch 256 --streams 3 --launches 24 --queue 192 > gpurun_out/${T}_mask_${v}.log 2>&1 || exit 1
  echo mask $v $(grep frames gpurun_out/${T}_mask_${v}.log)
done
