# round 3af (2): longer overlapped-bench A/B of the table sort, alternating order
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --kernel-pass 1 > gpurun_out/r3af2_radix_$r.log 2>&1 || exit 1
SSF_LIB=$L/libssf_frontend_bit.so timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --kernel-pass 1 > gpurun_out/r3af2_bit_$r.log 2>&1 || exit 1
done && echo AB_OK
