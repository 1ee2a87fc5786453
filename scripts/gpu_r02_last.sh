# Round 2, last: the GPU suite and smoke on the final library, then the
# profile recipe (stats, PMC traffic, SQ pass, bench line reading them).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02last}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
RUN=${RUN:-r02last}/prof bash scripts/gpu_r02_profile.sh > $O/profile.log 2>&1
rc=$?; echo RC=$rc; tail -1 $O/gpu_tests.log; tail -1 $O/smoke.log; tail -3 $O/profile.log | cut -c1-300; exit $rc
