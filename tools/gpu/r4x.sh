# round 4x: configs[2] with Kabsch warm starts -- kernel timelines (start / end per dispatch) for
# the automatic split (G = 8) and G = 1 over 4 mask streams, to see what serialises the step
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
K="$R/bench.py --consecutive 32 --kabsch-warm-start --steps 6 --warmup 2 --no-cpu-baseline --kernel-pass 0"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/r4x_a -o k -- python3 $K > $R/gpurun_out/r4x_auto.json 2> $R/gpurun_out/r4x_auto.err && \
cp $(find /tmp/r4x_a -name "*kernel_trace.csv" | head -1) $R/gpurun_out/r4x_auto_trace.csv && echo A && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/r4x_b -o k -- python3 $K --mask-split 1 --mask-streams 4 > $R/gpurun_out/r4x_g1s4.json 2> $R/gpurun_out/r4x_g1s4.err && \
cp $(find /tmp/r4x_b -name "*kernel_trace.csv" | head -1) $R/gpurun_out/r4x_g1s4_trace.csv && echo B
