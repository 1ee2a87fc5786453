# Round 4: C2 (N = 1) under other long-subject thresholds (bench.py
# --long-threshold; default 2,048 on C2), alternated twice.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r04sweep_lt}
mkdir -p $O
for rep in 1 2; do
  for lt in 0 1536 3072 4096; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify --sustained-seconds 0 --no-reference-scoring --long-threshold $lt > $O/lt${lt}_$rep.json 2> $O/lt${lt}_$rep.err || { echo "lt $lt FAILED"; tail -20 $O/lt${lt}_$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/lt${lt}_$rep.json').read().strip().split(chr(10))[-1])
print('lt', $lt, $rep, d['value'], d['ms_per_step'], d['config']['long_threshold'], d['config']['long_subjects_rank0'])"
  done
done
