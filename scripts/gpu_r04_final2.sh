# Round 4, last GPU step on HEAD: the GPU suite, smoke, then the profile
# script (kernel traces, PMC traffic and SQ pass of the current kernel
# sources, the bench line that reads them).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r04final2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
RUN=${RUN:-r04final2}/prof bash scripts/gpu_r04_profile.sh
