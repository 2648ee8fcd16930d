# round 4bc: final-build lines of the remaining configs (configs[4] 256k-pt scans, f64 inputs,
# edges, configs[2] 32 sequences, latency)
set -o pipefail
mkdir -p gpurun_out
T=r4bc
NB="--no-cpu-baseline"
timeout -k 10 400 python -u bench.py --n-az 4000 --steps 20 --warmup 3 $NB > gpurun_out/${T}_c5.json 2>/dev/null && echo C5 && \
timeout -k 10 400 python -u bench.py --f64-inputs --steps 20 --warmup 3 $NB > gpurun_out/${T}_f64in.json 2>/dev/null && echo F64 && \
timeout -k 10 400 python -u bench.py --edges --steps 20 --warmup 3 $NB > gpurun_out/${T}_edges.json 2>/dev/null && echo EDGES && \
timeout -k 10 300 python -u bench.py --mask-before-features --batch 32 --steps 30 --warmup 5 $NB > gpurun_out/${T}_c3b32.json 2>/dev/null && echo C3B32 && \
timeout -k 10 300 python -u bench.py --latency $NB > gpurun_out/${T}_lat.json 2>/dev/null && echo LAT
