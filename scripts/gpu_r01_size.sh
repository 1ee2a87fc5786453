# Scan-only GCUPS vs database size (fixed costs / tail), fp16 affine default.
set -o pipefail
O=gpurun_out/size; mkdir -p $O
for n in 570000 1140000 2280000; do
  SW_TUNE_SCORING=1:12:1 timeout -k 10 300 python3 scripts/tune_inter.py f32x8 2048,3072,1536 P07327 $n > $O/n$n.jsonl 2> $O/n$n.err || exit 1
done
echo RC=0; for f in $O/*.jsonl; do echo "== $f"; python3 -c "
import json
for l in open('$f'):
    d=json.loads(l); print(d['variant'], d['long_threshold'], d['n_long'], d['inter_ms'], d['intra_ms'], d['scan_ms'], d['gcups_scan'])
"; done
