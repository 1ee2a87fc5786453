# Packed two-subjects-per-lane kernel (x2): parity, then C2 sweeps.
set -o pipefail
O=gpurun_out/x2; mkdir -p $O
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/parity.log 2>&1 && \
for w in 386 640 1024 0; do
  SW_COOP_WIDTH=$w SW_TUNE_SCORING=1:12:1 timeout -k 10 300 python3 scripts/tune_inter.py x16x8,x16x16,x24x8,32x8 2048,1536,1024 > $O/aff_w$w.jsonl 2> $O/aff_w$w.err || exit 1
done && \
for w in 386 1024; do
  SW_COOP_WIDTH=$w timeout -k 10 300 python3 scripts/tune_inter.py x16x8,x16x16,x24x8,64x8 2048,1536 > $O/lin_w$w.jsonl 2> $O/lin_w$w.err || exit 1
done
rc=$?; echo RC=$rc; tail -3 $O/parity.log; for f in $O/*.jsonl; do echo "== $f"; cut -c1-62,100-240 $f; done; exit $rc
