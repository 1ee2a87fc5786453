# Round-end check: the whole GPU suite, smoke, the default bench line, and
# C4 with all 50M subjects on one GPU.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 900 python3 bench.py --config c4 --steps 3 --warmup 1 --no-reference-scoring > $O/c4_full.json 2> $O/c4_full.err
rc=$?; echo RC=$rc; tail -1 $O/parity.log; tail -1 $O/smoke.log
for f in bench c4_full; do [ -f $O/$f.json ] && python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f', d['value'], d['ms_per_step'], d['kernels'], r.get('value'), d.get('cpu_baseline',{}).get('value'), d['roofline'].get('traffic'), d.get('valu_roofline',{}).get('frac'))"; done; exit $rc
