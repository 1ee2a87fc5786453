# v19: biased fp16 cell in the intra kernel (sw_intra_x2): parity, C5, C2.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v19
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline > $O/c5.json 2> $O/c5.err && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; echo RC=$rc; tail -3 $O/parity.log; for f in c5 bench; do python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); print('$f', d['value'], d['kernel_ms_per_scan'], d.get('kernels'))"; done; exit $rc
