# Round 2: hardware-queue sharing (C3 under the reference scoring lost its
# int16 side launch's concurrency): exchange stream at high priority (its own
# queue pool) vs priority 0; C3 and the share of 8.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02y}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-verify"
timeout -k 10 300 $B --config c3 > $O/c3.json 2> $O/c3.err && \
timeout -k 10 300 $B --config c3 --exchange-priority 0 > $O/c3p0.json 2> $O/c3p0.err && \
timeout -k 10 300 $B --shard-of 8 > $O/s8.json 2> $O/s8.err && \
timeout -k 10 300 $B > $O/c2.json 2> $O/c2.err
rc=$?; echo RC=$rc; for f in $O/*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d.get('reference_scoring') or {}; print('$f', d['value'], d['ms_per_step'], '| ref', r.get('value'), r.get('kernel_ms_per_scan'))"; done; exit $rc
