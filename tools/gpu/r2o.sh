set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2o_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python -u bench.py > gpurun_out/r2o_bench.log 2>&1 && echo BENCH_OK
