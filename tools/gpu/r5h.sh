# round 5h: every GPU test + smoke on the run-kernel build; the default, carla and f64 lines; rocprof serial carla
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r5h
RX="--kernel-include-regex k_"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 400 python -u bench.py --layout carla --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_carla.json 2> gpurun_out/${T}_carla.err && echo CARLA_OK && \
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_default.json 2> gpurun_out/${T}_default.err && echo DEFAULT_OK && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats $RX --output-format csv -d /tmp/ps -o s -- python -u bench.py --layout carla --serial --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_carla_serial.log 2>&1 && echo SERIAL_OK && \
cp $(find /tmp/ps -name "*kernel_stats.csv" | head -1) gpurun_out/${T}_carla_serial_kernel_stats.csv
