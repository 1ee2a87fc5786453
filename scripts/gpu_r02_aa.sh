# Round 2: side streams created with the handle again (hardware-queue
# sharing), exchange stream at high priority: C3, C2, share of 8, GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02aa}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-verify"
timeout -k 10 300 $B --config c3 > $O/c3.json 2> $O/c3.err && \
timeout -k 10 300 $B --shard-of 8 > $O/s8.json 2> $O/s8.err && \
timeout -k 10 300 $B > $O/c2.json 2> $O/c2.err && \
timeout -k 10 300 $B --config c5 > $O/c5.json 2> $O/c5.err && \
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo RC=$rc; tail -2 $O/pytest.log; for f in $O/*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d.get('reference_scoring') or {}; print('$f', d['value'], d['ms_per_step'], '| ref', r.get('value'), r.get('ms_per_step'))"; done; exit $rc
