# round 6x: where k_plane_table_sorted's time goes -- timing-only builds that drop one part each
# (xfin: no plane fit, xrank: no rank walk, x2nd: no second pick walk, xdef: no deferred queries,
# xall: all four); outputs of these builds are NOT valid tables
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6x
L=$PWD/ssf-slam_amd/ssf/_lib
for rep in 1 2; do
for v in def xfin xrank x2nd xdef xall; do
  if [ $v = def ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python3 -u tools/bench_table.py > gpurun_out/${T}_${v}_$rep.log 2>&1 || { tail gpurun_out/${T}_${v}_$rep.log; exit 1; }
  echo $v $(tail -1 gpurun_out/${T}_${v}_$rep.log)
done
done
