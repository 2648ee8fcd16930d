# round 3v: EM pass split at B = 1 (diag stamps) + a second default bench for box variance
set -o pipefail
mkdir -p gpurun_out
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_mask_phases.py 1 > gpurun_out/r3v_phases_b1.log 2>&1 && echo PH1_OK && \
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 200 python -u tools/diag_mask_phases.py 256 > gpurun_out/r3v_phases_b256.log 2>&1 && echo PH256_OK && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3v_bench.log 2>&1 && echo BENCH_OK
