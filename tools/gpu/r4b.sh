# round 4b: configs[3] strong-scaling mode (N=1 line, N=2 one-GPU rehearsal), Kabsch warm start
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_registration.py -x -v --timeout 120 --timeout-method thread -k "kabsch_warm or per_step" > gpurun_out/r4b_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 7 --warmup 1 --no-cpu-baseline > gpurun_out/r4b_c4_n1.json 2> gpurun_out/r4b_c4_n1.err && echo C4N1_OK && \
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 7 --warmup 1 --kabsch-warm-start --no-cpu-baseline > gpurun_out/r4b_c4_n1_kws.json 2> gpurun_out/r4b_c4_n1_kws.err && echo C4KWS_OK && \
timeout -k 10 300 python -u bench.py --consecutive 32 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r4b_c3.json 2> gpurun_out/r4b_c3.err && echo C3_OK && \
timeout -k 10 300 python -u bench.py --consecutive 32 --steps 10 --warmup 2 --kabsch-warm-start --no-cpu-baseline > gpurun_out/r4b_c3_kws.json 2> gpurun_out/r4b_c3_kws.err && echo C3KWS_OK && \
timeout -k 10 400 python -u bench.py --gpus 2 --sequences-total 8 --consecutive 32 --steps 7 --warmup 1 --rehearse-one-gpu --no-cpu-baseline > gpurun_out/r4b_c4_n2_rehearse.json 2> gpurun_out/r4b_c4_n2_rehearse.err && echo C4N2_OK
