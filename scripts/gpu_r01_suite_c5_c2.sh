# Full GPU suite, C5 and C2 bench lines into gpurun_out/$RUN (default v25).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-v25}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline > $O/c5.json 2> $O/c5.err && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/c2.json 2> $O/c2.err
rc=$?; echo RC=$rc; tail -3 $O/parity.log; for f in c5 c2; do python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f', d['value'], d['kernels'], d['kernel_ms_per_scan'], r.get('value'), r.get('kernel_ms_per_scan'))"; done; exit $rc
