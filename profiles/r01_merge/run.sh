# Pair + single-wave blocks in one launch (SW_PAIR_MERGED=1, default) vs two
# concurrent launches; widths 256/512/1024; affine (f32x8) and linear (y32x8).
set -o pipefail
O=gpurun_out/merge; mkdir -p $O
timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "intra_two or inter_variants or pair or fp16_guard or default_kernel or batch" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for m in 1 0; do for w in 256 512 1024; do
  SW_PAIR_MERGED=$m SW_PAIR_WIDTH=$w SW_TUNE_SCORING=1:12:1 timeout -k 10 300 python3 scripts/tune_inter.py f32x8,f32x8 2048,3072 P07327 570000 > $O/aff_m${m}_w$w.jsonl 2> $O/aff_m${m}_w$w.err || { tail $O/aff_m${m}_w$w.err; exit 1; }
  SW_PAIR_MERGED=$m SW_PAIR_WIDTH=$w timeout -k 10 300 python3 scripts/tune_inter.py y32x8,y32x8 2048 P07327 570000 > $O/lin_m${m}_w$w.jsonl 2> $O/lin_m${m}_w$w.err || { tail $O/lin_m${m}_w$w.err; exit 1; }
done; done
for f in $O/*.jsonl; do echo "== $f"; python3 -c "
import json
for l in open('$f'):
    d=json.loads(l); print(d['variant'], d['long_threshold'], d['n_long'], d['inter_ms'], d['intra_ms'], d['scan_ms'], d['gcups_scan'])
"; done
