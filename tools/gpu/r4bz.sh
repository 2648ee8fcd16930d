# round 4bz: the final build's no-flag line as the driver runs it (traffic r04by), the configs[4]
# and latency lines
set -o pipefail
mkdir -p gpurun_out
T=r4bz
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_default_noflags.json 2> gpurun_out/${T}_default_noflags.err && echo NOFLAGS && \
timeout -k 10 400 python -u bench.py --n-az 4000 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_c5.json 2>/dev/null && echo C5 && \
timeout -k 10 300 python -u bench.py --latency --no-cpu-baseline > gpurun_out/${T}_lat.json 2>/dev/null && echo LAT
