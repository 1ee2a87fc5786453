# Round 3: the GPU suite (one pytest process, per-test timeout), then smoke().
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r03suite}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/gpu_tests.log; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; cat $O/smoke.log; exit 1; }
tail -1 $O/gpu_tests.log; cat $O/smoke.log
