set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py tests/test_gpu_nodes.py tests/test_gpu_features.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pick_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/pick_tests.log
for i in 1 2; do
timeout -k 10 200 python -u _ab_head/tools/bench_features.py --chain --distinct 256 --reps 5 --dump /tmp/pk_head.npz > gpurun_out/pk_head_$i.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_features.py --chain --distinct 256 --reps 5 --dump /tmp/pk_cur.npz > gpurun_out/pk_cur_$i.log 2>&1 || exit 1
done
python tools/cmp_npz.py /tmp/pk_head.npz /tmp/pk_cur.npz > gpurun_out/pk_cmp.log 2>&1
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_table_phases.py 256 > gpurun_out/pk_tphase.log 2>&1
