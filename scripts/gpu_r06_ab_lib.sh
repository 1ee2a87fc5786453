# Round 6 A/B of an alternative build ($B, same sources, other defines)
# against the tree's library: the GPU parity tests matching $K on $B first,
# then C2 (both scorings), its 1/8 share and $CFGS alternated $REPS times.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06ablib}
mkdir -p $O
SW_AMD_LIB=$B timeout -k 10 500 python -u -m pytest tests -x -q -m gpu -k "${K:-c2_size or merged_lpt or golden or tri_groups or tail_pipelined}" --timeout 300 --timeout-method thread > $O/b_tests.log 2>&1 || { echo B TESTS FAILED; tail -40 $O/b_tests.log; exit 1; }
tail -1 $O/b_tests.log
for rep in $(seq 1 ${REPS:-2}); do
  for v in tree alt; do
    lib=ece1782-smith-waterman-cuda_amd/lib/libswamd.so
    [ $v = alt ] && lib=$B
    for c in ${CFGS:-c2 s8}; do
      case $c in
        s8) args="--shard-of 8 --shard-rank 2" ;;
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
echo RC=0
