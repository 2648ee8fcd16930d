# round 4bp: hardware queues x mask streams in the default pipeline, alternating, 30 steps
# (the mask alone gains from a 4th stream, the pipeline with 4 HW queues did not: r04bn / r04bo)
set -o pipefail
mkdir -p gpurun_out
T=r4bp
B="python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline"
for i in 1 2; do
  timeout -k 10 200 $B > gpurun_out/${T}_q4s3_$i.json 2> gpurun_out/${T}_q4s3_$i.err && echo q4s3-$i || exit 1
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $B > gpurun_out/${T}_q8s3_$i.json 2> gpurun_out/${T}_q8s3_$i.err && echo q8s3-$i || exit 1
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $B --mask-streams 4 > gpurun_out/${T}_q8s4_$i.json 2> gpurun_out/${T}_q8s4_$i.err && echo q8s4-$i || exit 1
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $B --mask-streams 5 > gpurun_out/${T}_q8s5_$i.json 2> gpurun_out/${T}_q8s5_$i.err && echo q8s5-$i || exit 1
done
