# round 4bk: every config's line on the final build (k_feat_wave_reg both ways; traffic r04bj):
# the no-flag default line with the CPU legs, configs[4], f64 inputs, edges, configs[2] (32
# sequences; as written chained and with Kabsch warm starts), configs[3] (N = 1 chained / Kabsch
# warm starts, N = 2 one-GPU rehearsal), latency, smoke
set -o pipefail
mkdir -p gpurun_out
T=r4bk
NB="--no-cpu-baseline"
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_default_noflags.json 2> gpurun_out/${T}_default_noflags.err && echo DEF && \
timeout -k 10 400 python -u bench.py --n-az 4000 --steps 20 --warmup 3 $NB > gpurun_out/${T}_c5.json 2>/dev/null && echo C5 && \
timeout -k 10 400 python -u bench.py --f64-inputs --steps 20 --warmup 3 $NB > gpurun_out/${T}_f64in.json 2>/dev/null && echo F64 && \
timeout -k 10 400 python -u bench.py --edges --steps 20 --warmup 3 $NB > gpurun_out/${T}_edges.json 2>/dev/null && echo EDGES && \
timeout -k 10 300 python -u bench.py --mask-before-features --batch 32 --steps 30 --warmup 5 $NB > gpurun_out/${T}_c3b32.json 2>/dev/null && echo C3B32 && \
timeout -k 10 200 python -u bench.py --consecutive 32 --steps 30 --warmup 5 $NB > gpurun_out/${T}_c3.json 2>/dev/null && echo C3 && \
timeout -k 10 200 python -u bench.py --consecutive 32 --steps 30 --warmup 5 --kabsch-warm-start $NB > gpurun_out/${T}_c3kws.json 2>/dev/null && echo C3KWS && \
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 12 --warmup 5 $NB > gpurun_out/${T}_c4.json 2>/dev/null && echo C4 && \
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 12 --warmup 5 --kabsch-warm-start $NB > gpurun_out/${T}_c4kws.json 2>/dev/null && echo C4KWS && \
timeout -k 10 400 python -u bench.py --gpus 2 --sequences-total 8 --consecutive 32 --steps 12 --warmup 5 --rehearse-one-gpu $NB > gpurun_out/${T}_c4n2.json 2>/dev/null && echo C4N2 && \
timeout -k 10 300 python -u bench.py --latency $NB > gpurun_out/${T}_lat.json 2>/dev/null && echo LAT && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && echo SMOKE_OK
