set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_mask.py --batch 256 --splits 1,2,3,4 --reps 3 --distinct 256 > gpurun_out/r2b_split.log 2>&1
