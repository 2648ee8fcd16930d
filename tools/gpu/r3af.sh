# round 3af: plane-table sort by rocPRIM block radix sort vs the bitonic network (A/B)
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3af_pytest.log 2>&1 && echo PYTEST_OK && \
for r in 1 2; do
SSF_LIB=$L/libssf_frontend_bit.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --kernel-pass 5 > gpurun_out/r3af_bit_$r.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --kernel-pass 5 > gpurun_out/r3af_radix_$r.log 2>&1 || exit 1
done && echo AB_OK && \
timeout -k 10 300 python -u bench.py --latency --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r3af_latency.log 2>&1 && echo LAT_OK
