set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/parity3.log 2>&1 && \
timeout -k 10 600 python scripts/tune_inter.py > gpurun_out/tune1.jsonl 2> gpurun_out/tune1.err
rc=$?; echo RC=$rc; tail -2 gpurun_out/parity3.log; cat gpurun_out/tune1.jsonl; tail -3 gpurun_out/tune1.err; exit $rc
