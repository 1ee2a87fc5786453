# Round 3 A/B: single-wave blocks at widths rounded to 8 columns (default)
# against 16 (SW_BLK_COLS16=1), after the GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-s3c8}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
run() { tag=$1; shift; env "$@" timeout -k 10 600 python3 bench.py $ARGS > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$tag', d['value'], d['ms_per_step'], r.get('value'), d.get('parity_sample_ok'))"; }
for rep in 1 2; do
  ARGS="--no-cpu-baseline"; run c2_c8_$rep X=1; run c2_c16_$rep SW_BLK_COLS16=1
  ARGS="--no-cpu-baseline --shard-of 8"; run s8_c8_$rep X=1; run s8_c16_$rep SW_BLK_COLS16=1
  ARGS="--no-cpu-baseline --shard-of 4"; run s4_c8_$rep X=1; run s4_c16_$rep SW_BLK_COLS16=1
done
ARGS="--no-cpu-baseline --config c3"; run c3_c8 X=1; run c3_c16 SW_BLK_COLS16=1
