# round 4bh: k_feat_wave_reg (one wave per chunk, streamed column blocks, no barrier) against
# k_feat_chunk_reg (default build; the new kernel is variant wavereg, through SSF_LIB): parity of the feature / config / edge / node /
# registration tests, kernel-only feature times (alternating), rocprofv3 stats of the serial
# kernel pass, the default line
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r4bh
L=$GRAFT_REPO_ROOT/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_wavereg.so timeout -k 10 500 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_nodes.py tests/test_gpu_registration.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
for i in 1 2; do
  for v in wavereg default; do
    if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
    SSF_LIB=$lib timeout -k 10 120 python -u tools/bench_features.py --reps 5 --tag $v > gpurun_out/${T}_${v}_$i.json 2>&1 || exit 1
  done
done
echo FEAT_OK
SSF_LIB=$L/libssf_frontend_wavereg.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex k_ --output-format csv -d /tmp/ps -o s -- python -u bench.py --serial --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_serial_bench.log 2>&1 && echo SERIAL_OK && \
cp $(find /tmp/ps -name "*kernel_stats.csv" | head -1) gpurun_out/${T}_serial_kernel_stats.csv && \
SSF_LIB=$L/libssf_frontend_wavereg.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_def.json 2> gpurun_out/${T}_def.err && echo DEF
