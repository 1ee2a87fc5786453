# fp16 packed kernel: parity (incl. guard band / rescue chain), then C2 sweeps.
set -o pipefail
O=gpurun_out/fp16; mkdir -p $O
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/parity.log 2>&1 && \
SW_TUNE_SCORING=1:12:1 timeout -k 10 300 python3 scripts/tune_inter.py f32x8,y32x8,f32x8,y32x8 2048 > $O/aff.jsonl 2> $O/aff.err && \
timeout -k 10 300 python3 scripts/tune_inter.py y48x4,y32x4,y32x8,y48x4 2048 > $O/lin.jsonl 2> $O/lin.err && \
SW_TUNE_SCORING=1:12:1 timeout -k 10 300 python3 scripts/tune_inter.py f32x8,y32x8 2048 Q9UKN1 570000 > $O/aff_q9.jsonl 2> $O/aff_q9.err
rc=$?; echo RC=$rc; tail -3 $O/parity.log; for f in $O/*.jsonl; do echo "== $f"; python3 -c "
import json,sys
for l in open('$f'):
    d=json.loads(l); print(d['variant'], d['long_threshold'], d['ok'], d['inter_ms'], d['intra_ms'], d['gcups_scan'])
"; done; exit $rc
