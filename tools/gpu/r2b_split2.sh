set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_mask.py tests/test_gpu_configs.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/split_tests.log 2>&1 && \
timeout -k 10 200 python -u _ab_head/tools/bench_mask.py --batch 32 --splits 1,8 --reps 3 --distinct 32 > gpurun_out/split_head.log 2>&1 && \
timeout -k 10 200 python -u tools/bench_mask.py --batch 32 --splits 1,2,4,8 --reps 3 --distinct 32 > gpurun_out/split_cur.log 2>&1 && \
timeout -k 10 200 python -u tools/bench_mask.py --batch 256 --splits 1 --reps 3 --distinct 256 >> gpurun_out/split_cur.log 2>&1
