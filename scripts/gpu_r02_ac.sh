# Round 2: the merged launch with 16-row strips (3 workgroups per CU):
# its parity tests, then the share of 8 / 4 A/B on one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02ad}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-verify"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -k merged_lpt -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 $B --shard-of 8 > $O/s8_r32.json 2> $O/s8_r32.err && \
SW_LPT_ROWS=16 timeout -k 10 300 $B --shard-of 8 > $O/s8_r16.json 2> $O/s8_r16.err && \
timeout -k 10 300 $B --shard-of 8 > $O/s8_r32b.json 2> $O/s8_r32b.err && \
SW_LPT_ROWS=16 timeout -k 10 300 $B --shard-of 8 > $O/s8_r16b.json 2> $O/s8_r16b.err && \
timeout -k 10 300 $B --shard-of 4 > $O/s4_r32.json 2> $O/s4_r32.err && \
SW_LPT_ROWS=16 timeout -k 10 300 $B --shard-of 4 > $O/s4_r16.json 2> $O/s4_r16.err
rc=$?; echo RC=$rc; tail -2 $O/pytest.log; for f in $O/*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d.get('reference_scoring') or {}; print('$f', d['value'], d['ms_per_step'], '| ref', r.get('value'), r.get('ms_per_step'))"; done; exit $rc
