# Round 2: the linear biased cell in the intra kernel — GPU suite, then C5,
# C2 and the 1/8 share under both scorings, with and without it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02k}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
run() { tag=$1; shift; timeout -k 10 300 env "$@" python3 bench.py --no-verify --no-cpu-baseline $BARGS > $O/$tag.json 2> $O/$tag.err || exit 1; }
BARGS="--config c5"; run c5_lin; run c5_nolin SW_INTRA_LIN=0
BARGS=""; run c2_lin; run c2_nolin SW_INTRA_LIN=0
BARGS="--shard-of 8"; run s8_lin; run s8_nolin SW_INTRA_LIN=0
echo RC=0; tail -2 $O/tests.log
for f in $O/*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['kernels'], 'ref', r.get('value'), r.get('ms_per_step'), r.get('intra_kernel'), r.get('kernel_ms_per_scan',{}).get('sw_intra'))"; done
