# Small-db routing: parity, then C5 and C2 bench lines.
set -o pipefail
O=gpurun_out/route; mkdir -p $O
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/parity.log 2>&1 && \
timeout -k 10 600 python3 bench.py --config c5 > $O/c5.json 2> $O/c5.err && \
timeout -k 10 600 python3 bench.py --no-cpu-baseline > $O/c2.json 2> $O/c2.err
rc=$?; echo RC=$rc; tail -2 $O/parity.log; for f in c5 c2; do python3 -c "
import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms_per_scan'], d.get('reference_scoring',{}).get('value'), d.get('cpu_baseline'))"; done; exit $rc
