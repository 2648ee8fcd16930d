# round 3u (2): configs[2] consecutive line + default bench with the strip image reuse
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --consecutive 32 --batch 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3u_consec.json 2> gpurun_out/r3u_consec.err && echo CONSEC_OK && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3u_bench.log 2>&1 && echo BENCH_OK && \
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_mask_phases.py 1 > gpurun_out/r3u_phases_b1.log 2>&1 && echo PH1_OK
