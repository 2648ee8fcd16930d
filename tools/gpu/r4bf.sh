# round 4bf: 4-byte Lloyd records (SSF_LLOYD_REC4) -- mask parity tests on the variant, identical
# outputs on a 256-frame batch, mask launch times and the default line, alternating
set -o pipefail
mkdir -p gpurun_out
T=r4bf
L=$PWD/ssf-slam_amd/ssf/_lib
SSF_LIB=$L/libssf_frontend_rec4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_mask.py tests/test_gpu_configs.py tests/test_gpu_nodes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_rec4.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest_rec4.log; exit 1; }
for i in 1 2; do
  for v in default rec4; do
    if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
    SSF_LIB=$lib timeout -k 10 200 python -u tools/bench_mask.py --batch 256 --splits 1 --reps 3 --dump gpurun_out/${T}_dump_$v.npz > gpurun_out/${T}_mask_${v}_$i.json 2>&1 || exit 1
  done
done
python - <<'PY' && echo SAME
import numpy as np
a = np.load("gpurun_out/r4bf_dump_default.npz"); b = np.load("gpurun_out/r4bf_dump_rec4.npz")
for k in a.files:
    x, y = a[k], b[k]
    if k == "out":   # column 25 counts the streamed bytes (record size differs by design)
        x = np.delete(x, 25, axis=1); y = np.delete(y, 25, axis=1)
    assert np.array_equal(x, y), k
PY
for v in default rec4; do
  if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_def_$v.json 2>/dev/null || exit 1
done
echo ALL_OK
