# Round 2: hardware-queue assignment of the exchange stream (share of 8):
# lazily created side/copy streams, exchange stream priority, more queues.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02r}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-verify"
timeout -k 10 300 $B --shard-of 8 > $O/s8.json 2> $O/s8.err && \
timeout -k 10 300 $B --shard-of 8 --exchange-priority -1 > $O/s8p.json 2> $O/s8p.err && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 $B --shard-of 8 > $O/s8q.json 2> $O/s8q.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-verify --no-reference-scoring --shard-of 8 --steps 30 --exchange-priority -1 > $O/kt.json 2> $O/kt.err && \
timeout -k 10 300 $B > $O/c2.json 2> $O/c2.err
rc=$?; echo RC=$rc; grep -h "host enqueue" $O/*.err; for f in $O/*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('value_reference_scoring'))"; done; exit $rc
