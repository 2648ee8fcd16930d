set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/as_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/as_tests.log
for i in 1 2; do
timeout -k 10 200 python -u _ab_head/tools/bench_features.py --chain --distinct 256 --reps 5 --dump /tmp/as_head.npz > gpurun_out/as_head_$i.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_features.py --chain --distinct 256 --reps 5 --dump /tmp/as_cur.npz > gpurun_out/as_cur_$i.log 2>&1 || exit 1
done
python tools/cmp_npz.py /tmp/as_head.npz /tmp/as_cur.npz > gpurun_out/as_cmp.log 2>&1
timeout -k 10 200 python -u _ab_head/tools/bench_features.py --chain --distinct 256 --reps 3 --n-az 4000 --dump /tmp/as_head5.npz > gpurun_out/as_head5.log 2>&1 && \
timeout -k 10 200 python -u tools/bench_features.py --chain --distinct 256 --reps 3 --n-az 4000 --dump /tmp/as_cur5.npz > gpurun_out/as_cur5.log 2>&1 && \
python tools/cmp_npz.py /tmp/as_head5.npz /tmp/as_cur5.npz >> gpurun_out/as_cmp.log 2>&1
