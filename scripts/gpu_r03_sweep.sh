# Round 3: bench lines under environment overrides, one per line of $SWEEP
# ("tag VAR=value ... -- bench args"), all on one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r03sweep}
mkdir -p $O
while read -r tag rest; do
  [ -z "$tag" ] && continue
  envs="${rest%%--*}"; args="${rest#*--}"
  env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify --no-reference-scoring $args > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().split(chr(10))[-1])
print('$tag', d['value'], d['ms_per_step'], d.get('kernel_ms_per_scan',{}).get('scan_total'), d['config'].get('long_threshold'))"
done <<< "$SWEEP"
