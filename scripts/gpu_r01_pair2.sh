# Wave-pair kernel, narrower widths (down to every block) x long threshold on C2.
set -o pipefail
O=gpurun_out/pair2; mkdir -p $O
for w in 16 128 256 384 512; do
  SW_PAIR_WIDTH=$w SW_TUNE_SCORING=1:12:1 timeout -k 10 300 python3 scripts/tune_inter.py f32x8 2048,3072,4096,8192 P07327 570000 > $O/w$w.jsonl 2> $O/w$w.err || { tail $O/w$w.err; exit 1; }
  echo "w=$w done"
done
for f in $O/w*.jsonl; do echo "== $f"; python3 -c "
import json
for l in open('$f'):
    d=json.loads(l); print(d['variant'], d['long_threshold'], d['n_long'], d['inter_ms'], d['intra_ms'], d['scan_ms'], d['gcups_scan'])
"; done
