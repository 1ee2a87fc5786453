# Round 2: the wave-group passes and the merged launch's single-wave blocks
# with 8-row profile chunks (no register spills: scratch 148 -> 0 bytes):
# share of 8, C2, C3, then the GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02x}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-verify"
timeout -k 10 300 $B --shard-of 8 > $O/s8.json 2> $O/s8.err && \
timeout -k 10 300 $B > $O/c2.json 2> $O/c2.err && \
timeout -k 10 300 $B --config c3 > $O/c3.json 2> $O/c3.err && \
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo RC=$rc; tail -3 $O/pytest.log; for f in $O/*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('value_reference_scoring'), d.get('kernel_ms_per_scan'))"; done; exit $rc
