# C2: wave-pair width 1024 (default) vs 1536, alternating three times.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pairw2
mkdir -p $O
B="python3 bench.py --no-cpu-baseline"
for i in 1 2 3; do
  timeout -k 10 300 $B > $O/d$i.json 2> $O/d$i.err || exit $?
  SW_PAIR_WIDTH=1536 timeout -k 10 300 $B > $O/w$i.json 2> $O/w$i.err || exit $?
done
for f in d1 w1 d2 w2 d3 w3; do python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d['reference_scoring']
print('$f', d['value'], r['value'])"; done
