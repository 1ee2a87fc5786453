# Wave-pair kernel: parity first, then the C2 width x long-threshold sweep, then the full GPU suite.
set -o pipefail
O=gpurun_out/pair; mkdir -p $O
timeout -k 10 400 python3 -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "pair or fp16_guard or default_kernel" > $O/pytest_pair.log 2>&1 || { tail -30 $O/pytest_pair.log; exit 1; }
tail -2 $O/pytest_pair.log
for w in 0 512 768 1024 1536; do
  SW_PAIR_WIDTH=$w SW_TUNE_SCORING=1:12:1 timeout -k 10 300 python3 scripts/tune_inter.py f32x8 2048,3072,4096 P07327 570000 > $O/w$w.jsonl 2> $O/w$w.err || { tail $O/w$w.err; exit 1; }
  echo "w=$w done"
done
for f in $O/w*.jsonl; do echo "== $f"; python3 -c "
import json
for l in open('$f'):
    d=json.loads(l); print(d['variant'], d['long_threshold'], d['n_long'], d['inter_ms'], d['intra_ms'], d['scan_ms'], d['gcups_scan'])
"; done
timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > $O/pytest_all.log 2>&1 || { tail -30 $O/pytest_all.log; exit 1; }
tail -2 $O/pytest_all.log
