# round 4bo: the pipeline with 3 (default) against 4 and 5 mask streams, alternating, 30 steps
# (mask alone: 64.4 k frames/s on 3 streams, 66.7 k on 4, r04bn)
set -o pipefail
mkdir -p gpurun_out
T=r4bo
for i in 1 2; do
  for m in 3 4 5; do
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --mask-streams $m > gpurun_out/${T}_ms${m}_$i.json 2> gpurun_out/${T}_ms${m}_$i.err && echo ms$m-$i || exit 1
  done
done
