set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_mask.py --batch 256 --splits 1,2,3,4 --distinct 64 > gpurun_out/r2n_mask.log 2>&1 && echo M_OK && \
for sp in 1 2 4; do timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --mask-split $sp --distinct 64 > gpurun_out/r2n_bench_s$sp.log 2>&1 || exit 1; done && echo BENCH_OK && \
for sp in 2 4; do timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --mask-split $sp --distinct 64 --mask-streams 1 > gpurun_out/r2n_bench_s${sp}_ms1.log 2>&1 || exit 1; done && echo BENCH1_OK && \
timeout -k 10 300 python -u bench.py --mask-before-features --batch 32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r2n_bench_c3.log 2>&1 && echo C3_OK
