# round 3b: k_curv_select probes (greedy / stencil cost), features tests, BatchScanner vs synth.scan
set -o pipefail
mkdir -p gpurun_out
L=$PWD/ssf-slam_amd/ssf/_lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3b_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 200 python -u tools/diag_synth.py > gpurun_out/r3b_synth.json 2> gpurun_out/r3b_synth.err && echo SYNTH_OK && \
for n in frontend cp1 cp2 frontend; do f=libssf_frontend_$n.so; [ $n = frontend ] && f=libssf_frontend.so; SSF_LIB=$L/$f timeout -k 10 200 python -u tools/bench_features.py --tag $n --reps 10 >> gpurun_out/r3b_probe.log 2>&1 || exit 1; done && echo PROBE_OK
