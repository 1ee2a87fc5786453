# Round 6: the N-rank exchange's device work rehearsed beside the share's scans
# (bench.py --shard-of 8 --rehearse-exchange: each step's device top-100, a
# one-rank RCCL all-gather, 7 more rows copied in and the device merge of
# 8 x 100 keys, all on the exchange stream beside the next scan), against the
# same share without it, alternating, for the slowest rank (2) and rank 0,
# both scorings in each line, C2 on the same box first and last.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06exchange}
mkdir -p $O
b() { tag=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu-baseline --sustained-seconds 0 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -20 $O/$tag.err; exit 1; }; tail -1 $O/$tag.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('reference_scoring',{}); print('$tag', d['value'], d['ms_per_step'], r.get('value'), d.get('parity_sample_ok'), bool(d.get('exchange_rehearsed')))"; }
b c2_first
for rep in 1 2; do
  for k in 2 0; do
    b s8_r${k}_plain_$rep --shard-of 8 --shard-rank $k
    b s8_r${k}_xchg_$rep --shard-of 8 --shard-rank $k --rehearse-exchange
  done
done
b c2_last
echo RC=0
