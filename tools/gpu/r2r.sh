set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RX="--kernel-include-regex k_"
timeout -k 10 400 rocprofv3 --kernel-trace --stats $RX --output-format csv -d /tmp/ps -o s -- python -u bench.py --serial --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r2r_serial_bench.log 2>&1 && echo SERIAL_OK && \
cp $(find /tmp/ps -name "*kernel_stats.csv" | head -1) gpurun_out/r2r_serial_kernel_stats.csv && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats $RX --output-format csv -d /tmp/pd -o d -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2r_default_bench.log 2>&1 && echo DEFAULT_OK && \
cp $(find /tmp/pd -name "*kernel_stats.csv" | head -1) gpurun_out/r2r_default_kernel_stats.csv && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats $RX --output-format csv -d /tmp/p5 -o f -- python -u bench.py --serial --n-az 4000 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/r2r_c5_serial_bench.log 2>&1 && echo C5_OK && \
cp $(find /tmp/p5 -name "*kernel_stats.csv" | head -1) gpurun_out/r2r_c5_serial_kernel_stats.csv
du -sh gpurun_out
