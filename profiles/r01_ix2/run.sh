# Packed two-subjects intra kernel: parity, C5 bench packed vs int32, C2 pair-width x threshold sweep.
set -o pipefail
O=gpurun_out/ix2; mkdir -p $O
timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "intra_two or inter_variants or pair or fp16_guard" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 bench.py --config c5 --steps 5 --warmup 1 > $O/c5_x2.json 2> $O/c5_x2.err || { tail $O/c5_x2.err; exit 1; }
SW_INTRA_X2=0 timeout -k 10 300 python3 bench.py --config c5 --steps 5 --warmup 1 > $O/c5_i32.json 2> $O/c5_i32.err || { tail $O/c5_i32.err; exit 1; }
python3 -c "
import json
for f in ['c5_x2','c5_i32']:
    d=json.loads(open('$O/'+f+'.json').read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d.get('kernel'), d.get('roofline',{}).get('frac'))
"
for w in 16 256 512; do
  SW_PAIR_WIDTH=$w SW_TUNE_SCORING=1:12:1 timeout -k 10 300 python3 scripts/tune_inter.py f32x8 1024,2048,3072,4096 P07327 570000 > $O/w$w.jsonl 2> $O/w$w.err || { tail $O/w$w.err; exit 1; }
done
for f in $O/w*.jsonl; do echo "== $f"; python3 -c "
import json
for l in open('$f'):
    d=json.loads(l); print(d['variant'], d['long_threshold'], d['n_long'], d['inter_ms'], d['intra_ms'], d['scan_ms'], d['gcups_scan'])
"; done
