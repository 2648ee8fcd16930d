# round 6zl: timing experiment -- the features stream without the two fallback launches
# (k_feat_wave_run, k_feat_chunk_flagged; nofb, valid only when k_feat_wave_reg leaves them no
# chunk, as on the azimuth bench frames) vs the final build: default line at 60 steps, alternating
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r6zl
L=$PWD/ssf-slam_amd/ssf/_lib
for rep in 1 2 3; do
for v in def nofb; do
  if [ $v = def ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_${v}_$rep.json 2> gpurun_out/${T}_${v}_$rep.err || { tail -5 gpurun_out/${T}_${v}_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d.get('stage_event_ms'))" gpurun_out/${T}_${v}_$rep.json $v
done
done
