# round 4z: the plane table's queries split over up to 8 work-groups per frame for small batches:
# parity (registration, configs, nodes, features), then latency, configs[2] and the default line
set -o pipefail
mkdir -p gpurun_out
T=r4z
timeout -k 10 500 python -u -m pytest tests/test_gpu_registration.py tests/test_gpu_configs.py tests/test_gpu_nodes.py tests/test_gpu_edges.py tests/test_examples.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
timeout -k 10 200 python -u bench.py --latency --no-cpu-baseline > gpurun_out/${T}_latency.json 2> gpurun_out/${T}_latency.err && echo LAT && \
timeout -k 10 200 python -u bench.py --consecutive 32 --kabsch-warm-start --steps 10 --warmup 2 --no-cpu-baseline --timeline > gpurun_out/${T}_c3kws.json 2> gpurun_out/${T}_c3kws.err && echo KWS && \
timeout -k 10 200 python -u bench.py --consecutive 32 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err && echo C3 && \
timeout -k 10 200 python -u bench.py --mask-before-features --batch 32 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_c3b32.json 2> gpurun_out/${T}_c3b32.err && echo C3B32 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_def.json 2> gpurun_out/${T}_def.err && echo DEF
