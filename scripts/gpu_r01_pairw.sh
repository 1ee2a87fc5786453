# C2 with the wave-pair width threshold swept (after chained passes).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pairw
mkdir -p $O
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 300 $B > $O/def.json 2> $O/def.err || exit $?
for w in 512 768 1536 2048 4096; do
  SW_PAIR_WIDTH=$w timeout -k 10 300 $B > $O/w$w.json 2> $O/w$w.err || exit $?
done
timeout -k 10 300 $B > $O/def2.json 2> $O/def2.err || exit $?
for f in def w512 w768 w1536 w2048 w4096 def2; do python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d['reference_scoring']
print('$f', d['value'], d['kernel_ms_per_scan']['sw_inter'], r['value'])"; done
