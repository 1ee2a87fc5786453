# Round 4 measurement: (the GPU suite unless NOSUITE=1), smoke, the default bench line (C2,
# N=1), the strong-scaling shares, bench.py --gpus 2 launching its own two
# ranks (gloo, both on this GPU), C1, C3, C4 (one rank's share of 8) and C5.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r04round}
mkdir -p $O
[ -n "$NOSUITE" ] || timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; cat $O/smoke.log; exit 1; }
b() { tag=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -5 $O/$tag.err; exit 1; }; }
b c2
b c2_share2 --shard-of 2
b c2_share4 --shard-of 4
b c2_share8 --shard-of 8
b c2_2rank_self --gpus 2 --backend gloo --device 0
b c1 --config c1
b c3 --config c3
b c4_share8 --config c4 --shard-of 8 --steps 5 --warmup 1
b c5 --config c5
echo RC=0; [ -n "$NOSUITE" ] || tail -1 $O/gpu_tests.log; cat $O/smoke.log
for f in c2 c2_share2 c2_share4 c2_share8 c2_2rank_self c1 c3 c4_share8 c5; do python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f', d['n_gpus'], d['value'], d['ms_per_step'], d.get('kernels'), r.get('value'), d.get('cpu_baseline',{}).get('value'), d.get('cpu_baseline',{}).get('one_thread'), d.get('parity_sample_ok'), (d.get('parity') or {}).get('whole_database'), d.get('valu_roofline',{}) and d['valu_roofline'].get('frac'), (d.get('sustained') or {}).get('value'))"; done
