# Round 2: same-box A/B of eager vs first-use side streams on the share of 8
# and C3 (hardware-queue sharing).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02ac}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-verify"
timeout -k 10 300 $B --shard-of 8 > $O/s8_eager.json 2> $O/s8_eager.err && \
SW_LAZY_STREAMS=1 timeout -k 10 300 $B --shard-of 8 > $O/s8_lazy.json 2> $O/s8_lazy.err && \
timeout -k 10 300 $B --shard-of 8 > $O/s8_eager2.json 2> $O/s8_eager2.err && \
SW_LAZY_STREAMS=1 timeout -k 10 300 $B --shard-of 8 > $O/s8_lazy2.json 2> $O/s8_lazy2.err
rc=$?; echo RC=$rc; for f in $O/*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d.get('reference_scoring') or {}; print('$f', d['value'], d['ms_per_step'], '| ref', r.get('value'), r.get('ms_per_step'))"; done; exit $rc
