# round 4bd: k_solve threads per pair for few pairs (latency line B = 1; configs[2] chained B = 1)
set -o pipefail
mkdir -p gpurun_out
T=r4bd
L=$PWD/ssf-slam_amd/ssf/_lib
for v in default sv512 sv1024; do
  if [ $v = default ]; then lib=$L/libssf_frontend.so; else lib=$L/libssf_frontend_$v.so; fi
  SSF_LIB=$lib timeout -k 10 200 python -u bench.py --latency --no-cpu-baseline > gpurun_out/${T}_lat_$v.json 2>/dev/null || exit 1
  SSF_LIB=$lib timeout -k 10 200 python -u bench.py --consecutive 32 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_c3_$v.json 2>/dev/null || exit 1
done
echo ALL_OK
