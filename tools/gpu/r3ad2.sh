set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
for c in "256 1" "1 32"; do set -- $c
SSF_LIB=$L/libssf_frontend_m2.so timeout -k 10 200 python -u tools/dump_mask.py $1 $2 gpurun_out/r3ad_m2_$1.npz > gpurun_out/r3ad2_dump.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/dump_mask.py $1 $2 gpurun_out/r3ad_mw_$1.npz >> gpurun_out/r3ad2_dump.log 2>&1 || exit 1
python tools/cmp_npz.py gpurun_out/r3ad_m2_$1.npz gpurun_out/r3ad_mw_$1.npz >> gpurun_out/r3ad2_cmp.log && rm -f gpurun_out/r3ad_m2_$1.npz gpurun_out/r3ad_mw_$1.npz || exit 1
done
echo CMP_OK
