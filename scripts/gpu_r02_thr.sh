# Round 2: the 1/8 share of C2 over the long threshold (the library's default
# scales it with the database: ~900 here), plus the quad width.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02thr}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-verify --no-reference-scoring --shard-of 8"
for t in 0 700 800 1000 1200; do
  timeout -k 10 300 $B --long-threshold $t > $O/s8_t$t.json 2> $O/s8_t$t.err || exit 1
done
for w in 450 800; do
  SW_QUAD_WIDTH=$w timeout -k 10 300 $B > $O/s8_q$w.json 2> $O/s8_q$w.err || exit 1
done
timeout -k 10 300 $B > $O/s8_t0b.json 2> $O/s8_t0b.err || exit 1
for f in $O/*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print('$f', d['value'], d['ms_per_step'], c.get('long_threshold'), c.get('long_subjects_rank0'))"; done
