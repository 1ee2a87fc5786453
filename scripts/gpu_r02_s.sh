# Round 2: fewer packets between scans (events recorded only where read,
# repeated readbacks skipped, lazily created streams): GPU suite, share of 8,
# C2, and a kernel trace of the share.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02s}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-verify"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 $B --shard-of 8 > $O/s8.json 2> $O/s8.err && \
timeout -k 10 300 $B --shard-of 8 --exchange-priority -1 > $O/s8p.json 2> $O/s8p.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-verify --no-reference-scoring --shard-of 8 --steps 30 > $O/kt.json 2> $O/kt.err && \
timeout -k 10 300 $B > $O/c2.json 2> $O/c2.err
rc=$?; echo RC=$rc; tail -3 $O/pytest.log; grep -h "host enqueue" $O/*.err; for f in $O/*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('kernel_ms_per_scan'))"; done; exit $rc
