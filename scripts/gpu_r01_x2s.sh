# Two-strips-per-lane packed kernel (yRxSG): parity, then C2 sweeps.
set -o pipefail
O=gpurun_out/x2s2; mkdir -p $O
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/parity.log 2>&1 && \
SW_COOP_WIDTH=0 SW_TUNE_SCORING=1:12:1 timeout -k 10 300 python3 scripts/tune_inter.py y32x8,y32x4,y16x8 2048,3072,4096 > $O/aff_w0.jsonl 2> $O/aff_w0.err && \
SW_COOP_WIDTH=1536 SW_TUNE_SCORING=1:12:1 timeout -k 10 300 python3 scripts/tune_inter.py y32x8,y32x4 3072,4096 > $O/aff_w1536.jsonl 2> $O/aff_w1536.err && \
SW_COOP_WIDTH=0 timeout -k 10 300 python3 scripts/tune_inter.py 64x8,y32x8,y32x4,y48x4 2048,3072 > $O/lin_w0.jsonl 2> $O/lin_w0.err && \
SW_COOP_WIDTH=386 timeout -k 10 300 python3 scripts/tune_inter.py 64x8,y32x4,y48x4 2048 > $O/lin_w386.jsonl 2> $O/lin_w386.err
rc=$?; echo RC=$rc; tail -3 $O/parity.log; for f in $O/*.jsonl; do echo "== $f"; python3 -c "
import json,sys
for l in open('$f'):
    d=json.loads(l); print(d['variant'], d['long_threshold'], d['n_long'], d['inter_ms'], d['intra_ms'], d['gcups_scan'])
"; done; exit $rc
