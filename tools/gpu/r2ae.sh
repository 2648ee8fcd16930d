set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2ae_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 200 python -u tools/bench_features.py --tag strips_table --reps 5 --chain > gpurun_out/r2ae_feat.log 2>&1 && echo FEAT_OK && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2ae_bench.log 2>&1 && echo BENCH_OK && \
timeout -k 10 400 python -u bench.py --n-az 4000 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r2ae_bench_c5.log 2>&1 && echo BENCH5_OK
