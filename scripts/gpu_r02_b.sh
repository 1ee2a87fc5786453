# Round 2: the C2/8 share (one rank of 8, strong scaling) vs the long
# threshold and the wave-pair width; then the trimmed library's GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02b}
mkdir -p $O
for t in 512 704 1024 1536; do
  timeout -k 10 200 python3 bench.py --shard-of 8 --no-reference-scoring --no-verify --long-threshold $t > $O/s8_t$t.json 2> $O/s8_t$t.err || exit 1
done
for pw in 128 64; do
  SW_PAIR_WIDTH=$pw timeout -k 10 200 python3 bench.py --shard-of 8 --no-reference-scoring --no-verify --long-threshold 704 > $O/s8_t704_pw$pw.json 2> $O/s8_t704_pw$pw.err || exit 1
done
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/parity.log 2>&1
rc=$?; echo RC=$rc; tail -3 $O/parity.log
for f in $O/s8_*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().split(chr(10))[-1])
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d.get('kernel_ms_per_scan'), d['config']['long_subjects_rank0'])"; done; exit $rc
