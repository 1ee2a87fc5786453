# Round 6: C1 (BASELINE configs[0], CPU path + the GPU on the same database)
# and C4 (configs[3], one rank's 6.25M-subject share generated in HBM) on the
# round-6 sources, with their parity legs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06c14}
mkdir -p $O
timeout -k 10 600 python3 bench.py --config c1 > $O/c1.json 2> $O/c1.err || { echo C1 FAILED; tail -10 $O/c1.err; exit 1; }
tail -1 $O/c1.json | cut -c1-300
for k in ${C4RANKS:-0 7}; do
  timeout -k 10 600 python3 bench.py --config c4 --shard-of 8 --shard-rank $k --no-cpu-baseline > $O/c4_share8_r$k.json 2> $O/c4_share8_r$k.err || { echo C4 FAILED; tail -10 $O/c4_share8_r$k.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/c4_share8_r$k.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('c4 r$k', d['value'], d['ms_per_step'], r.get('value'), d.get('parity_sample_ok'), d['parity']['subjects_checked'], r.get('parity_ok'))"
done
echo RC=0
