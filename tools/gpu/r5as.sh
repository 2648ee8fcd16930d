# round 5as: --edges with the edge cloud / line table in the step ring: allocator growth in the
# timed region, and the edge tests
set -o pipefail
mkdir -p gpurun_out
T=r5as
timeout -k 10 500 python -u -m pytest tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
timeout -k 10 600 python -u bench.py --edges --steps 30 --no-cpu-baseline > gpurun_out/${T}_edges.json 2> gpurun_out/${T}_edges.err || { tail -20 gpurun_out/${T}_edges.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_edges.json').read().strip().splitlines()[-1]);print('edges', round(d['value']), d['allocator_timed_region'])"
