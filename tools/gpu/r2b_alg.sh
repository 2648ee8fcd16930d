set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_mask.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/alg_tests.log 2>&1 && \
for i in 1 2; do
timeout -k 10 200 python -u _ab_head/tools/bench_mask.py --batch 256 --splits 1 --reps 3 --distinct 256 --dump gpurun_out/alg_head.npz > gpurun_out/alg_head_$i.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_mask.py --batch 256 --splits 1 --reps 3 --distinct 256 --dump gpurun_out/alg_cur.npz > gpurun_out/alg_cur_$i.log 2>&1 || exit 1
done
