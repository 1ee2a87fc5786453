# Round 4 A/B of two builds (lib = the tree's, $B = an alternative build of
# the same sources with other defines): the tests matching $FIRST on the
# tree's build, then the 1/8 share (both scorings) and $CFGS alternated twice.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r04ab}
mkdir -p $O
if [ -n "$FIRST" ]; then timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "$FIRST" --timeout 200 --timeout-method thread > $O/first_tests.log 2>&1 || { echo FIRST TESTS FAILED; tail -40 $O/first_tests.log; exit 1; }; tail -1 $O/first_tests.log; fi
for rep in 1 2; do
  for v in new old; do
    lib=ece1782-smith-waterman-cuda_amd/lib/libswamd.so
    [ $v = old ] && lib=$B
    for c in ${CFGS:-s8}; do
      case $c in
        s8) args="--shard-of 8" ;;
        c2) args="" ;;
        c5) args="--config c5" ;;
        c3) args="--config c3" ;;
      esac
      SW_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify --sustained-seconds 0 $args > $O/${c}_${v}_$rep.json 2> $O/${c}_${v}_$rep.err || { echo "$c $v FAILED"; tail -20 $O/${c}_${v}_$rep.err; exit 1; }
      python3 -c "
import json
d=json.loads(open('$O/${c}_${v}_$rep.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$c $v $rep', d['value'], d['ms_per_step'], r.get('value'), r.get('ms_per_step'))"
    done
  done
done
