# round 3al: overlapped bench with 2, 3, 4 mask streams (alternating order, 40 steps)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for ms in 3 4 2; do
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --kernel-pass 1 --mask-streams $ms > gpurun_out/r3al_ms${ms}_$r.log 2>&1 || exit 1
done; done && echo MS_OK
