# Round 6 check: the GPU suite, smoke(), the default bench line as the driver
# runs it, then (SHARES=1) scripts/gpu_r06_shares.sh into the same directory.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06check}
mkdir -p $O
if [ -z "$NOSUITE" ]; then timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/gpu_tests.log; exit 1; }; tail -1 $O/gpu_tests.log; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ -z "$NOBENCH" ]; then timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH FAILED; tail -20 $O/bench_default.err; exit 1; }; tail -1 $O/bench_default.json | cut -c1-400; fi
if [ -n "$SHARES" ]; then RUN=${RUN:-r06check} bash scripts/gpu_r06_shares.sh || exit 1; fi
echo RC=0
