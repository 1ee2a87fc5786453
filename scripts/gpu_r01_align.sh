# GPU traceback tests (+ full parity).
set -o pipefail
O=gpurun_out/align; mkdir -p $O
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/parity.log 2>&1
rc=$?; echo RC=$rc; tail -30 $O/parity.log; exit $rc
