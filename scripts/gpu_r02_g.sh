# Round 2: the merged longest-first launch (sw_scan_lpt): parity, then C2
# and its strong-scaling shares against the two-launch form.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02g}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo TESTS FAILED; tail -40 $O/parity.log; exit 1; }
run() { tag=$1; shift; timeout -k 10 200 env "$@" python3 bench.py --no-reference-scoring --no-verify $BARGS > $O/$tag.json 2> $O/$tag.err || exit 1; }
for sh in 8 4 2; do
  BARGS="--shard-of $sh"
  run s${sh}_lpt_g2 SW_PAIR_GROUP=2
  run s${sh}_lpt_g4 SW_PAIR_GROUP=4
  run s${sh}_lpt_g4_w64 SW_PAIR_GROUP=4 SW_PAIR_WIDTH=64
  run s${sh}_nolpt SW_LPT=0
done
BARGS=""
run c2_lpt_g2 SW_PAIR_GROUP=2
run c2_lpt_g4 SW_PAIR_GROUP=4
run c2_nolpt SW_LPT=0
echo RC=0; tail -2 $O/parity.log
for f in $O/*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().split(chr(10))[-1])
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['kernels']['inter'], d.get('kernel_ms_per_scan'), d['config']['long_subjects_rank0'], d['config']['long_threshold'])"; done
