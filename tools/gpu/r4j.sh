# round 4j: the default bench, new feature stage vs the round-3 stage (legacy library), alternating
# on one box; and the data dependence of the 8-sequence configs[3] shape (8 distinct sequences in
# the default shape)
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4j_pytest.log 2>&1 && echo PYTEST_OK || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/r4j_new_$i.json 2> gpurun_out/r4j_new_$i.err || exit 1
  SSF_LIB=$L/libssf_frontend_legacy.so timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/r4j_old_$i.json 2> gpurun_out/r4j_old_$i.err || exit 1
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --distinct 8 --no-cpu-baseline > gpurun_out/r4j_distinct8.json 2> gpurun_out/r4j_distinct8.err || exit 1
echo ALL_OK
