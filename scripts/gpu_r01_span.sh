# Widest blocks in int16 first (adaptive span): GPU suite, C3, C2.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/span
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/parity.log 2>&1 && \
B="python3 bench.py --no-cpu-baseline" && \
timeout -k 10 600 $B --config c3 > $O/c3.json 2> $O/c3.err && \
timeout -k 10 300 $B > $O/c2.json 2> $O/c2.err
rc=$?; echo RC=$rc; tail -3 $O/parity.log
for f in c3 c2; do [ -f $O/$f.json ] && python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f', d['value'], d['kernel_ms_per_scan'], r.get('value'), r.get('kernel'), r.get('kernel_ms_per_scan'))"; done; exit $rc
