# Round 5: the long threshold of C2's 1/8 share under both scorings (the
# share's span is its widest pair blocks' latency, which the threshold sets:
# profiles/r05_trace/).  Thresholds in $LTS (0 = the library's, 891 here),
# alternated $REPS times.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r05lt}
mkdir -p $O
B="bench.py --no-cpu-baseline --no-verify --sustained-seconds 0 --shard-of ${SHARD:-8}"
for rep in $(seq 1 ${REPS:-2}); do
  for lt in ${LTS:-0 650 750 1000}; do
    a=""; [ $lt != 0 ] && a="--long-threshold $lt"
    timeout -k 10 300 python3 $B $a > $O/s8_lt${lt}_$rep.json 2> $O/s8_lt${lt}_$rep.err || { echo "lt $lt FAILED"; tail -20 $O/s8_lt${lt}_$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/s8_lt${lt}_$rep.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('lt $lt $rep', d['value'], d['ms_per_step'], r.get('value'), r.get('ms_per_step'))"
  done
done
echo RC=0
