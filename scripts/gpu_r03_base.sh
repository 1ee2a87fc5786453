# Round 3 baseline: the default bench line, bench.py launching its own 2 ranks
# (gloo, both on this GPU), the 1/8 share.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r03base}
mkdir -p $O
b() { tag=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -20 $O/$tag.err; exit 1; }; }
b c2
b c2_2rank_self --gpus 2 --backend gloo --device 0
b c2_share8 --shard-of 8
b c2_share4 --shard-of 4
for f in c2 c2_2rank_self c2_share8 c2_share4; do python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f', d['n_gpus'], d['value'], d['ms_per_step'], d.get('kernels'), r.get('value'), d.get('parity_sample_ok'), (d.get('parity') or {}).get('whole_database'))"; done
