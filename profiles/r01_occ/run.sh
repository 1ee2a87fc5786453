# fp16 two-strips shapes: 32x8 (2 waves/SIMD), 32x4 with 8-row chunks (2 waves), forced 3 waves (g32x4, spills),
# 24x4 (3 waves); parity first, then C2 scan-only at long threshold 3072, pair kernel off.
set -o pipefail
O=gpurun_out/occ; mkdir -p $O
timeout -k 10 400 python3 -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "inter_variants and (f32x4 or f24x4 or g32x4 or f32x8)" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
SW_PAIR_WIDTH=0 SW_TUNE_SCORING=1:12:1 timeout -k 10 400 python3 scripts/tune_inter.py f32x8,f32x4,g32x4,f24x4 2048,3072 P07327 570000 > $O/occ.jsonl 2> $O/occ.err || { tail $O/occ.err; exit 1; }
python3 -c "
import json
for l in open('$O/occ.jsonl'):
    d=json.loads(l); print(d['variant'], d['long_threshold'], d['n_long'], d['inter_ms'], d['intra_ms'], d['scan_ms'], d['gcups_scan'])
"
