# round 4bs: the registration of step k waits for step k's features only (not its plane table):
# pose dumps of both orders compared bitwise, then alternating lines (default vs --reg-after-table)
set -o pipefail
mkdir -p gpurun_out
T=r4bs
B="python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline"
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --dump-poses gpurun_out/${T}_poses_new.npy > gpurun_out/${T}_dump_new.json 2>/dev/null && \
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --reg-after-table --dump-poses gpurun_out/${T}_poses_old.npy > gpurun_out/${T}_dump_old.json 2>/dev/null && \
python -c "
import numpy as np, sys
a = np.load('gpurun_out/${T}_poses_new.npy'); b = np.load('gpurun_out/${T}_poses_old.npy')
print('poses', a.shape, 'bit-identical', a.tobytes() == b.tobytes())
sys.exit(0 if a.tobytes() == b.tobytes() else 1)" > gpurun_out/${T}_poses_cmp.txt && echo POSES_OK || { cat gpurun_out/${T}_poses_cmp.txt; exit 1; }
for i in 1 2 3; do
  timeout -k 10 200 $B > gpurun_out/${T}_new_$i.json 2>/dev/null && echo new-$i || exit 1
  timeout -k 10 200 $B --reg-after-table > gpurun_out/${T}_old_$i.json 2>/dev/null && echo old-$i || exit 1
done
