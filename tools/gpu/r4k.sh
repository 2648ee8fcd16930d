# round 4k: is the configs[3] step slower because of its later frames (the synthetic street ends
# near x = 370 m; the ego moves ~1 m per frame)?  Same mode, frames <= 96 vs <= 256
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 2 --warmup 1 --kabsch-warm-start --no-cpu-baseline > gpurun_out/r4k_c4_s2.json 2> gpurun_out/r4k_c4_s2.err || exit 1
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 7 --warmup 1 --kabsch-warm-start --no-cpu-baseline > gpurun_out/r4k_c4_s7.json 2> gpurun_out/r4k_c4_s7.err || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 150 --kernel-pass 0 --batch 64 --no-cpu-baseline > gpurun_out/r4k_late_frames.json 2> gpurun_out/r4k_late_frames.err || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --kernel-pass 0 --batch 64 --no-cpu-baseline > gpurun_out/r4k_early_frames.json 2> gpurun_out/r4k_early_frames.err || exit 1
echo ALL_OK
