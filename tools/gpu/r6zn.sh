# round 6zn: the final labelling pass with its LDS parameter bases laundered once per pass (new:
# default build, SSF_FINAL_LDS_HOIST) vs per point (fh0 = the r06fin-final build): mask tests, the
# mask alone, then the default line at 60 steps, alternating
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6zn
L=$PWD/ssf-slam_amd/ssf/_lib
for v in new; do
  if [ $v = new ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_mask.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_$v.log 2>&1 && echo PYTEST_OK $v || { tail -20 gpurun_out/${T}_pytest_$v.log; exit 1; }
done
for rep in 1 2; do
for v in fh0 new; do
  if [ $v = new ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python3 -u tools/bench_mask_overlap.py --batch 256 --streams 3 --launches 24 --queue 192 > gpurun_out/${T}_mask_${v}_$rep.log 2>&1 || exit 1
  echo mask $v $(grep frames gpurun_out/${T}_mask_${v}_$rep.log)
done
done
for rep in 1 2 3; do
for v in fh0 new; do
  if [ $v = new ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_${v}_$rep.json 2> gpurun_out/${T}_${v}_$rep.err || { tail -5 gpurun_out/${T}_${v}_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['roofline']['frac'])" gpurun_out/${T}_${v}_$rep.json $v
done
done
