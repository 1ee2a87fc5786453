# Round 2: quads inside the merged launch — parity, then the shares against
# the quad width.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02i}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "lpt or wave_pair or saturation" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
run() { tag=$1; shift; timeout -k 10 200 env "$@" python3 bench.py --no-reference-scoring --no-verify $BARGS > $O/$tag.json 2> $O/$tag.err || exit 1; }
for sh in 8 4; do
  BARGS="--shard-of $sh"
  run s${sh}_q0 SW_QUAD_WIDTH=0
  run s${sh}_qdef
  run s${sh}_q300 SW_QUAD_WIDTH=300
  run s${sh}_q600 SW_QUAD_WIDTH=600
done
BARGS="--shard-of 8 --long-threshold 1024"; run s8_t1024_qdef
BARGS="--shard-of 8 --long-threshold 1024"; run s8_t1024_q500 SW_QUAD_WIDTH=500
BARGS="--shard-of 8 --long-threshold 900"; run s8_t900_qdef
echo RC=0; tail -2 $O/tests.log
for f in $O/*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().split(chr(10))[-1])
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['kernels']['inter'], d.get('kernel_ms_per_scan')['scan_total'], d['config']['long_subjects_rank0'], d['config']['long_threshold'])"; done
