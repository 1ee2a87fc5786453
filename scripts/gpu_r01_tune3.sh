set -o pipefail
mkdir -p gpurun_out
V=${1:-64x8,k16x8,k32x8,k16x16,k32x4}
T=${2:-1536}
SW_INTER_VARIANT=k16x8 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/parity_t3a.log 2>&1 && \
SW_INTER_VARIANT=k32x8 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/parity_t3b.log 2>&1 && \
timeout -k 10 600 python scripts/tune_inter.py $V $T > gpurun_out/tune3.jsonl 2> gpurun_out/tune3.err
rc=$?; echo RC=$rc; tail -3 gpurun_out/parity_t3a.log; tail -3 gpurun_out/parity_t3b.log; cat gpurun_out/tune3.jsonl; tail -3 gpurun_out/tune3.err; exit $rc
