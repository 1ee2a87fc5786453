# Column-skewed inter kernels: parity over every variant, then C2 sweeps
# (affine BLOSUM62 12/1 and linear BLOSUM50 2), coop skew on/off.
set -o pipefail
O=gpurun_out/skew; mkdir -p $O
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/parity.log 2>&1 && \
for sk in 1 0; do
  SW_COOP_SKEW=$sk SW_TUNE_SCORING=1:12:1 timeout -k 10 300 python3 scripts/tune_inter.py 32x8,s32x8,32x16,s32x16,16x16,s16x16,s48x8 2048,1536 > $O/aff_sk$sk.jsonl 2> $O/aff_sk$sk.err || exit 1
  SW_COOP_SKEW=$sk timeout -k 10 300 python3 scripts/tune_inter.py 64x8,s64x8,s32x8,s48x8,s32x16 2048,1536 > $O/lin_sk$sk.jsonl 2> $O/lin_sk$sk.err || exit 1
done
rc=$?; echo RC=$rc; tail -2 $O/parity.log; for f in $O/*.jsonl; do echo "== $f"; cut -c1-62,100-240 $f; done; exit $rc
