# Round 2: profiles copied on their own stream (overlapping the running
# scan) — GPU suite, then C2 and the shares.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02p}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
run() { tag=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -5 $O/$tag.err; exit 1; }; }
run c2
run s8 --shard-of 8
run s4 --shard-of 4 --no-reference-scoring
run s2 --shard-of 2 --no-reference-scoring
run c3 --config c3 --no-reference-scoring
echo RC=0; tail -2 $O/tests.log
for f in $O/*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d.get('kernel_ms_per_scan')['scan_total'], r.get('value'), r.get('ms_per_step'))" 2>/dev/null; done
