set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
true && \
for i in 1 2; do
timeout -k 10 200 python -u _ab_head/tools/bench_features.py --chain --distinct 256 --reps 5 --dump /tmp/defer_head.npz > gpurun_out/defer_head_$i.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_features.py --chain --distinct 256 --reps 5 --dump /tmp/defer_cur.npz > gpurun_out/defer_cur_$i.log 2>&1 || exit 1
done && \
timeout -k 10 200 python -u _ab_head/tools/bench_features.py --chain --distinct 256 --reps 3 --n-az 4000 --dump /tmp/defer_head5.npz > gpurun_out/defer_head5.log 2>&1 && \
timeout -k 10 200 python -u tools/bench_features.py --chain --distinct 256 --reps 3 --n-az 4000 --dump /tmp/defer_cur5.npz > gpurun_out/defer_cur5.log 2>&1
python tools/cmp_npz.py /tmp/defer_head.npz /tmp/defer_cur.npz > gpurun_out/defer_cmp.log 2>&1
python tools/cmp_npz.py /tmp/defer_head5.npz /tmp/defer_cur5.npz >> gpurun_out/defer_cmp.log 2>&1
