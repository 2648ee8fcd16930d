# round 6t: EM with two point pairs in flight (emd2) vs one (default): mask-only throughput
# (3 streams, queue 192), alternating; golden mask tests on the variant
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6t
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_emd2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mask.py -x -q --timeout 120 --timeout-method thread -k "golden or full_size or schedule" > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -20 gpurun_out/${T}_pytest.log; exit 1; }
for rep in 1 2 3; do
for v in def emd2; do
  if [ $v = def ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python3 -u tools/bench_mask_overlap.py --batch 256 --streams 3 --launches 24 --queue 192 > gpurun_out/${T}_${v}_$rep.log 2>&1 || exit 1
  echo $v $(grep frames gpurun_out/${T}_${v}_$rep.log)
done
done
