# round 6u: EM point pairs staged by LDS-DMA (emd4: parameters from LDS, emd4s: parameters in
# SGPRs), SGPR parameters alone (ems), the unrolled swap form (emd3) vs the default:
# golden mask tests per variant, then mask-only throughput (3 streams, queue 192), alternating
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6u
L=$PWD/ssf-slam_amd/ssf/_lib
for v in emd4s emd4 ems emd3; do
  SSF_LIB=$L/libssf_frontend_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mask.py -x -q --timeout 120 --timeout-method thread -k "golden or full_size or schedule" > gpurun_out/${T}_pytest_$v.log 2>&1 && echo PYTEST_OK $v || { tail -20 gpurun_out/${T}_pytest_$v.log; exit 1; }
done
for rep in 1 2; do
for v in def emd4s emd4 ems emd3; do
  if [ $v = def ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python3 -u tools/bench_mask_overlap.py --batch 256 --streams 3 --launches 24 --queue 192 > gpurun_out/${T}_${v}_$rep.log 2>&1 || exit 1
  echo $v $(grep frames gpurun_out/${T}_${v}_$rep.log)
done
done
