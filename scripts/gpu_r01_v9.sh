# v9 (re-entry after container re-creation): rebuilt libraries, full GPU
# parity suite, default bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v9
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo RC=$rc; tail -3 $O/parity.log; cut -c1-1500 $O/bench.json; tail -3 $O/bench.err; exit $rc
