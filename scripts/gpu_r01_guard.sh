# Guarded int16 (x2s + int32 rescue) for long queries: parity, then C3/C5-like timings.
set -o pipefail
O=gpurun_out/guard; mkdir -p $O
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/parity.log 2>&1 && \
for g in 1 0; do
  SW_INT16_GUARD=$g SW_TUNE_SCORING=1:12:1 timeout -k 10 300 python3 scripts/tune_inter.py y32x8 2048 Q9UKN1 570000 > $O/q9_g$g.jsonl 2> $O/q9_g$g.err || exit 1
  SW_INT16_GUARD=$g SW_TUNE_SCORING=1:12:1 timeout -k 10 300 python3 scripts/tune_inter.py y32x8 2048 P28167 570000 > $O/p28_g$g.jsonl 2> $O/p28_g$g.err || exit 1
done
rc=$?; echo RC=$rc; tail -3 $O/parity.log; for f in $O/*.jsonl; do echo "== $f"; cut -c1-300 $f; done; exit $rc
