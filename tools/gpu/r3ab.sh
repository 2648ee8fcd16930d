# round 3ab: overlapped bench with 1, 2, 4 work-groups per frame (MALL-sized working sets)
set -o pipefail
mkdir -p gpurun_out
for g in 1 2 4; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --mask-split $g --kernel-pass 1 > gpurun_out/r3ab_g$g.log 2>&1 || exit 1
echo G${g}_OK
done
