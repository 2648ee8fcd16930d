set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py tests/test_gpu_nodes.py tests/test_gpu_features.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sort_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/pick_tests.log
for i in 1 2; do
timeout -k 10 200 python -u _ab_head/tools/bench_features.py --chain --distinct 256 --reps 5 --dump /tmp/sr_head.npz > gpurun_out/sr_head_$i.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_features.py --chain --distinct 256 --reps 5 --dump /tmp/sr_cur.npz > gpurun_out/sr_cur_$i.log 2>&1 || exit 1
done
python tools/cmp_npz.py /tmp/sr_head.npz /tmp/sr_cur.npz > gpurun_out/sr_cmp.log 2>&1
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_table_phases.py 256 > gpurun_out/sr_tphase.log 2>&1
timeout -k 10 200 python -u _ab_head/tools/bench_features.py --chain --distinct 256 --reps 3 --n-az 4000 --dump /tmp/sr_head5.npz > gpurun_out/sr_head5.log 2>&1 && \
timeout -k 10 200 python -u tools/bench_features.py --chain --distinct 256 --reps 3 --n-az 4000 --dump /tmp/sr_cur5.npz > gpurun_out/sr_cur5.log 2>&1 && \
python tools/cmp_npz.py /tmp/sr_head5.npz /tmp/sr_cur5.npz >> gpurun_out/sr_cmp.log 2>&1
