# round 5b: k_feat_wave_run (channel-major / ragged runs) + the wave_reg probe column: feature GPU
# tests, the carla and default bench lines, rocprof of the serial carla and default runs
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r5b
RX="--kernel-include-regex k_"
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_edges.py tests/test_gpu_configs.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 400 python -u bench.py --layout carla --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_carla.json 2> gpurun_out/${T}_carla.err && echo CARLA_OK && \
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_default.json 2> gpurun_out/${T}_default.err && echo DEFAULT_OK && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats $RX --output-format csv -d /tmp/ps -o s -- python -u bench.py --layout carla --serial --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_carla_serial.log 2>&1 && echo SERIAL_OK && \
cp $(find /tmp/ps -name "*kernel_stats.csv" | head -1) gpurun_out/${T}_carla_serial_kernel_stats.csv && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats $RX --output-format csv -d /tmp/pd -o d -- python -u bench.py --serial --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_default_serial.log 2>&1 && echo SERIAL2_OK && \
cp $(find /tmp/pd -name "*kernel_stats.csv" | head -1) gpurun_out/${T}_default_serial_kernel_stats.csv
