# Round 4, after quads were limited to small databases: the GPU suite,
# smoke, C2 and its 1/2, 1/4, 1/8 shares, bench.py --gpus 2 on this GPU, then
# the profile script (kernel traces, PMC traffic and SQ pass of these
# kernel sources, the bench line that reads them).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r04final3}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
b() { tag=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$tag', d['n_gpus'], d['value'], d['ms_per_step'], r.get('value'), d.get('parity_sample_ok'), (d.get('sustained') or {}).get('value'))"; }
b c2
b c2_share2 --shard-of 2 --no-cpu-baseline
b c2_share4 --shard-of 4 --no-cpu-baseline
b c2_share8 --shard-of 8 --no-cpu-baseline
b c2_2rank_self --gpus 2 --backend gloo --device 0 --no-cpu-baseline
RUN=${RUN:-r04final3}/prof bash scripts/gpu_r04_profile.sh
