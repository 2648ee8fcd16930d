set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py tests/test_gpu_nodes.py tests/test_examples.py tests/test_gpu_edges.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2ab_tests.log 2>&1 && echo TESTS_OK && \
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_table_phases.py 256 > gpurun_out/r2ab_table.log 2>&1 && echo TABLE_OK && \
timeout -k 10 200 python -u tools/bench_features.py --tag strips_table --reps 5 --chain > gpurun_out/r2ab_feat.log 2>&1 && echo FEAT_OK && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2ab_bench.log 2>&1 && echo BENCH_OK && \
timeout -k 10 400 python -u bench.py --n-az 4000 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r2ab_bench_c5.log 2>&1 && echo BENCH5_OK
