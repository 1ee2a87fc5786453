# Round 5: progress counts published after the LDS operations only by ring
# feeders (SW_PAIR_PUBLISH_LDS=1: lib_pl, affine groups; lib_plall, every
# group) against the full workgroup release (the tree's lib).  The GPU suite
# on lib_plall, then C2 and its 1/8 and 1/4 shares alternated $REPS times.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r05pub}
mkdir -p $O
P=ece1782-smith-waterman-cuda_amd
SW_AMD_LIB=$P/lib_plall/libswamd.so timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests_plall.log 2>&1 || { echo TESTS FAILED; tail -40 $O/gpu_tests_plall.log; exit 1; }
tail -1 $O/gpu_tests_plall.log
RUN=${RUN:-r05pub} REPS=${REPS:-2} CFGS="${CFGS:-c2 s8 s4}" VARIANTS="base:- pl:lib_pl plall:lib_plall" bash scripts/gpu_r05_ab.sh
