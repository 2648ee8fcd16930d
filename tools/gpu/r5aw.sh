# round 5aw: the N = 2 paths on one GPU (gloo rehearsal): the default pipeline (weak scaling, one
# all-gather of the pose records at the end) and configs[3]'s strong mode, with this round's rings
set -o pipefail
mkdir -p gpurun_out
T=r5aw
timeout -k 10 600 python -u bench.py --gpus 2 --rehearse-one-gpu --steps 10 --warmup 2 --no-cpu-baseline --batch 64 > gpurun_out/${T}_n2.json 2> gpurun_out/${T}_n2.err || { tail -20 gpurun_out/${T}_n2.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_n2.json').read().strip().splitlines()[-1]);print('n2', round(d['value']), d['n_gpus'], d.get('gather_check'), d.get('allocator_timed_region'), d['config'].get('backend'))"
timeout -k 10 600 python -u bench.py --gpus 2 --rehearse-one-gpu --sequences-total 8 --consecutive 32 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c4n2.json 2> gpurun_out/${T}_c4n2.err || { tail -20 gpurun_out/${T}_c4n2.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_c4n2.json').read().strip().splitlines()[-1]);print('c4n2', round(d['value']), d['n_gpus'], d.get('gather_check'), d.get('allocator_timed_region'))"
