set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/parity_t4.log 2>&1 && \
SW_COOP_WIDTH=16 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/parity_t4b.log 2>&1 && \
for cw in 0 1024 768 512 384; do SW_COOP_WIDTH=$cw timeout -k 10 300 python scripts/tune_inter.py 64x8 1536,2048,3072 | sed "s/^/{\"coop\": $cw, \"r\": /;s/$/}/" ; done > gpurun_out/tune4.jsonl 2> gpurun_out/tune4.err
rc=$?; echo RC=$rc; tail -2 gpurun_out/parity_t4.log; tail -2 gpurun_out/parity_t4b.log; cat gpurun_out/tune4.jsonl; tail -3 gpurun_out/tune4.err; exit $rc
