# C5 with the intra kernel's rows per lane forced to 16 vs the cost model's
# choice (20 for a 5,000-aa query), and the intra parity tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ri
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k intra --timeout 120 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline > $O/c5_auto.json 2> $O/c5_auto.err && \
SW_INTRA_X2_RI=16 timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline > $O/c5_16.json 2> $O/c5_16.err
rc=$?; echo RC=$rc; tail -2 $O/parity.log; for f in c5_auto c5_16; do python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); print('$f', d['value'], d['kernels'], d['valu_roofline']['frac'], d.get('reference_scoring',{}).get('value'))"; done; exit $rc
