# x2 with 32-row strips (chunked profile reads): parity, then C2 BLOSUM62 12/1 sweeps.
set -o pipefail
O=gpurun_out/x2b; mkdir -p $O
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/parity.log 2>&1 && \
for w in 1024 1536 768; do
  SW_COOP_WIDTH=$w SW_TUNE_SCORING=1:12:1 timeout -k 10 300 python3 scripts/tune_inter.py x16x16,x32x8,x32x16,x48x8 2048,1536 > $O/aff_w$w.jsonl 2> $O/aff_w$w.err || exit 1
done
rc=$?; echo RC=$rc; tail -3 $O/parity.log; for f in $O/*.jsonl; do echo "== $f"; python3 -c "
import json,sys
for l in open('$f'):
    d=json.loads(l); print(d['variant'], d['long_threshold'], d['n_long'], d['inter_ms'], d['intra_ms'], d['gcups_scan'])
"; done; exit $rc
