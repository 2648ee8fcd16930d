# round 4n: the bench line of every config on the current build (one box)
set -o pipefail
mkdir -p gpurun_out
T=r4n
NB="--no-cpu-baseline"
timeout -k 10 300 python -u bench.py --consecutive 32 --steps 10 --warmup 2 $NB > gpurun_out/${T}_c3_consec.json 2> gpurun_out/${T}_c3_consec.err && echo C3_OK && \
timeout -k 10 300 python -u bench.py --consecutive 32 --steps 10 --warmup 2 --kabsch-warm-start $NB > gpurun_out/${T}_c3_consec_kws.json 2> gpurun_out/${T}_c3_consec_kws.err && echo C3KWS_OK && \
timeout -k 10 300 python -u bench.py --mask-before-features --batch 32 --steps 20 --warmup 3 $NB > gpurun_out/${T}_c3_b32.json 2> gpurun_out/${T}_c3_b32.err && echo C3B32_OK && \
timeout -k 10 400 python -u bench.py --n-az 4000 --steps 20 --warmup 3 $NB > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err && echo C5_OK && \
timeout -k 10 400 python -u bench.py --f64-inputs --steps 20 --warmup 3 $NB > gpurun_out/${T}_f64in.json 2> gpurun_out/${T}_f64in.err && echo F64IN_OK && \
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 7 --warmup 1 $NB > gpurun_out/${T}_c4_n1.json 2> gpurun_out/${T}_c4_n1.err && echo C4_OK && \
timeout -k 10 300 python -u bench.py --sequences-total 8 --consecutive 32 --steps 7 --warmup 1 --kabsch-warm-start $NB > gpurun_out/${T}_c4_n1_kws.json 2> gpurun_out/${T}_c4_n1_kws.err && echo C4KWS_OK && \
timeout -k 10 400 python -u bench.py --gpus 2 --sequences-total 8 --consecutive 32 --steps 7 --warmup 1 --rehearse-one-gpu $NB > gpurun_out/${T}_c4_n2_rehearse.json 2> gpurun_out/${T}_c4_n2_rehearse.err && echo C4N2_OK && \
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_default_noflags.json 2> gpurun_out/${T}_default_noflags.err && echo DEF_OK
