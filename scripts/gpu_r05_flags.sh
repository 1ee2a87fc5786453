# Round 5: flag-synchronised wave groups (SW_PAIR_FLAGS=1, lib_flags) against
# the tick-barrier form (the tree's lib): the GPU suite on lib_flags, then
# A/B of C2, its 1/8 and 1/4 shares, and wave groups on every block
# (SW_PAIR_WIDTH=16: the hand-off through LDS rings).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r05flags}
mkdir -p $O
P=ece1782-smith-waterman-cuda_amd
if [ -z "$NOSUITE" ]; then
  SW_AMD_LIB=$P/lib_flags/libswamd.so timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests_flags.log 2>&1 || { echo TESTS FAILED; tail -40 $O/gpu_tests_flags.log; exit 1; }
  tail -1 $O/gpu_tests_flags.log
fi
RUN=${RUN:-r05flags} REPS=${REPS:-2} CFGS="${CFGS:-c2 s8 s4}" VARIANTS="${VARIANTS:-tick:- flags:lib_flags tickall:-:SW_PAIR_WIDTH=16 flagsall:lib_flags:SW_PAIR_WIDTH=16}" bash scripts/gpu_r05_ab.sh
