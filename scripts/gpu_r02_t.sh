# Round 2: intra kernel stores lane 63's boundary column itself (no per-step
# cross-lane collection): GPU suite, C5 (affine and reference scoring), C2,
# share of 8.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02t}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-verify"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 $B --config c5 > $O/c5.json 2> $O/c5.err && \
timeout -k 10 300 $B > $O/c2.json 2> $O/c2.err && \
timeout -k 10 300 $B --shard-of 8 > $O/s8.json 2> $O/s8.err
rc=$?; echo RC=$rc; tail -3 $O/pytest.log; for f in $O/*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('value_reference_scoring'), d.get('kernel_ms_per_scan'))"; done; exit $rc
