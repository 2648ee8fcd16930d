# round 4bq: bench.py sets GPU_MAX_HW_QUEUES=8 by default (--hw-queues): alternating against the
# environment's 4 (--hw-queues 0) on the default line, configs[2] with Kabsch warm starts and the
# latency line; then the no-flag line as the driver runs it
set -o pipefail
mkdir -p gpurun_out
T=r4bq
NB="--no-cpu-baseline"
for i in 1 2 3; do
  for q in 8 0; do
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 $NB --hw-queues $q > gpurun_out/${T}_def_q${q}_$i.json 2>/dev/null && echo def-q$q-$i || exit 1
  done
done
for q in 8 0; do
  timeout -k 10 200 python -u bench.py --consecutive 32 --steps 30 --warmup 5 --kabsch-warm-start $NB --hw-queues $q > gpurun_out/${T}_c3kws_q$q.json 2>/dev/null && echo c3kws-q$q || exit 1
  timeout -k 10 200 python -u bench.py --latency $NB --hw-queues $q > gpurun_out/${T}_lat_q$q.json 2>/dev/null && echo lat-q$q || exit 1
  timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 12 --warmup 5 $NB --hw-queues $q > gpurun_out/${T}_c4_q$q.json 2>/dev/null && echo c4-q$q || exit 1
done
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_default_noflags.json 2> gpurun_out/${T}_default_noflags.err && echo NOFLAGS
