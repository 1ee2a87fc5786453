# Round 6: every rank's share of a strong-scaled C2, measured alone on one
# GPU (bench.py --shard-of N --shard-rank k) for N in $NS (default 8; "2 4 8"
# for all), both scorings in each line (the affine headline and the
# reference's BLOSUM50 / linear 2 under reference_scoring), with C2 itself
# (N = 1) on the same box first and last, then scripts/share_summary.py.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06shares}
mkdir -p $O
b() { tag=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu-baseline --sustained-seconds 0 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -20 $O/$tag.err; exit 1; }; tail -1 $O/$tag.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('reference_scoring',{}); print('$tag', d['value'], d['ms_per_step'], r.get('value'), d.get('parity_sample_ok'))"; }
b c2_first
for N in ${NS:-8}; do
  for k in $(seq 0 $((N - 1))); do b s${N}_r$k --shard-of $N --shard-rank $k; done
done
b c2_last
python3 scripts/share_summary.py $O > $O/summary.json && cat $O/summary.json
echo RC=0
