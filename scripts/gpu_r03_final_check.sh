# Round 3 closing check of HEAD: the GPU suite, smoke() and the default bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s3final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/c2.json 2> $O/c2.err || { echo BENCH FAILED; tail -5 $O/c2.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c2.json').read().strip().split(chr(10))[-1])
print(d['value'], d['ms_per_step'], d['roofline'].get('traffic'), d['roofline'].get('frac'), d.get('parity_sample_ok'), d['cpu_baseline']['value'])"
