# Device-generated shards: parity (incl. synthetic tests), then config C4 at
# one rank's share of 8 GPUs (6.25M subjects) and the whole 50M on one GPU.
set -o pipefail
O=gpurun_out/c4; mkdir -p $O
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/parity.log 2>&1 && \
timeout -k 10 600 python3 bench.py --config c4 --db-seqs 6250000 --steps 5 --warmup 1 > $O/c4_share8.json 2> $O/c4_share8.err && \
timeout -k 10 900 python3 bench.py --config c4 --steps 3 --warmup 1 --no-reference-scoring > $O/c4_full.json 2> $O/c4_full.err
rc=$?; echo RC=$rc; tail -2 $O/parity.log; for f in c4_share8 c4_full; do python3 -c "
import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d['config']['subjects_per_rank'], d['config']['residues_per_rank'], d['kernel_ms_per_scan'], d.get('reference_scoring',{}).get('value'), d.get('cpu_baseline'))" ; tail -3 $O/$f.err; done; exit $rc
