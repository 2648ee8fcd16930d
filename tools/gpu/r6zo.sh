# round 6zo: k_mask_pose at 512 threads (2 waves per SIMD, 256 VGPRs, 7 spilled; t512) vs 768
# (3 waves, 168 VGPRs, 87 spilled; new = the final build): mask tests on t512, the mask alone,
# then the default line at 60 steps, alternating
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6zo
L=$PWD/ssf-slam_amd/ssf/_lib
for v in t512; do
  if [ $v = new ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_mask.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_$v.log 2>&1 && echo PYTEST_OK $v || { tail -20 gpurun_out/${T}_pytest_$v.log; exit 1; }
done
for rep in 1 2; do
for v in t512 new; do
  if [ $v = new ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python3 -u tools/bench_mask_overlap.py --batch 256 --streams 3 --launches 24 --queue 192 > gpurun_out/${T}_mask_${v}_$rep.log 2>&1 || exit 1
  echo mask $v $(grep frames gpurun_out/${T}_mask_${v}_$rep.log)
done
done
for rep in 1 2 3; do
for v in t512 new; do
  if [ $v = new ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_${v}_$rep.json 2> gpurun_out/${T}_${v}_$rep.err || { tail -5 gpurun_out/${T}_${v}_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['roofline']['frac'])" gpurun_out/${T}_${v}_$rep.json $v
done
done
