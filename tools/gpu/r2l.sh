set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/probes/l3_stream > gpurun_out/r2l_l3.log 2>&1 && echo L3_OK && \
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_solvestamps.so timeout -k 10 120 python -u tools/bench_features.py --tag stamps --reps 2 --chain --stamps > gpurun_out/r2l_stamps.log 2>&1 && echo STAMPS_OK && \
SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 120 python -u tools/diag_table_phases.py 256 > gpurun_out/r2l_table.log 2>&1 && echo TABLE_OK && \
for B in 256 64 32; do SSF_LIB=$PWD/ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so timeout -k 10 120 python -u tools/diag_mask_phases.py $B >> gpurun_out/r2l_mask.log 2>&1 || exit 1; done && echo MASK_OK
