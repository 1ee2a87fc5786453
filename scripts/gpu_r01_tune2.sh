set -o pipefail
mkdir -p gpurun_out
V=${1:-64x8,p64x8,p64x4,p32x8,p48x8}
T=${2:-1536,1024}
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/parity_t2.log 2>&1 && \
SW_INTER_VARIANT=p64x8 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/parity_t2p.log 2>&1 && \
timeout -k 10 600 python scripts/tune_inter.py $V $T > gpurun_out/tune2.jsonl 2> gpurun_out/tune2.err
rc=$?; echo RC=$rc; tail -1 gpurun_out/parity_t2.log; tail -1 gpurun_out/parity_t2p.log; cat gpurun_out/tune2.jsonl; tail -3 gpurun_out/tune2.err; exit $rc
