# Farrar-form affine + affine cooperative kernel: parity, then C2 BLOSUM62
# 12/1 sweeps over shapes and coop widths (SW_COOP_WIDTH; 0 = off).
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/aff2; mkdir -p $O
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $O/parity.log 2>&1 && \
for w in 0 256 384 640 1024; do
  SW_COOP_WIDTH=$w SW_TUNE_SCORING=1:12:1 timeout -k 10 300 python3 scripts/tune_inter.py 32x8,32x16,16x16 2048,1536 > $O/w$w.jsonl 2> $O/w$w.err || exit 1
done
rc=$?; echo RC=$rc; tail -2 $O/parity.log; for w in 0 256 384 640 1024; do echo "== width $w"; cut -c1-60,100-240 $O/w$w.jsonl; done; exit $rc
