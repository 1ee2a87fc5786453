# Round 6: knob sweep on rank $SRANK's share of C2 at N = $SHARD (both
# scorings per line, no parity leg: timing only): long threshold x quad width
# (sw_opts quad_width via SW_QUAD_WIDTH) x pair width, then C2 itself.
# CASES: "tag:long_threshold:quad_width:pair_width:extra_env ..." (-1 =
# default).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06sweep}
mkdir -p $O
for c in ${CASES}; do
  IFS=: read tag lt qw pw ex <<< "$c"
  envs=""; [ "$qw" != "-1" ] && envs="$envs SW_QUAD_WIDTH=$qw"; [ "$pw" != "-1" ] && envs="$envs SW_PAIR_WIDTH=$pw"
  [ -n "$ex" ] && envs="$envs ${ex//,/ }"
  a=""; [ "$lt" != "-1" ] && a="--long-threshold $lt"
  env $envs timeout -k 10 300 python3 bench.py --shard-of ${SHARD:-8} --shard-rank ${SRANK:-2} --no-cpu-baseline --no-verify --sustained-seconds 0 --steps 200 $a > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$tag', '$envs', '$a', d['value'], d['ms_per_step'], r.get('value'), r.get('ms_per_step'), d['config']['long_threshold'], d['kernels']['inter'])"
done
echo RC=0
