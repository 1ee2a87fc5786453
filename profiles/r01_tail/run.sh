# Tail test: widest blocks to the (int32) cooperative kernel beside the fp16 kernel.
set -o pipefail
O=gpurun_out/tail; mkdir -p $O
for w in 0 1024 1536 768; do
  SW_COOP_WIDTH=$w SW_TUNE_SCORING=1:12:1 timeout -k 10 300 python3 scripts/tune_inter.py f32x8 2048,3072 P07327 570000 > $O/w$w.jsonl 2> $O/w$w.err || exit 1
done
echo RC=0; for f in $O/*.jsonl; do echo "== $f"; python3 -c "
import json
for l in open('$f'):
    d=json.loads(l); print(d['variant'], d['long_threshold'], d['n_long'], d['inter_ms'], d['intra_ms'], d['scan_ms'], d['gcups_scan'])
"; done
