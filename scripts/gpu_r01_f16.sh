# Packed fp16 (v_pk_maximum3_f16) vs packed int16 cell issue rates.
set -o pipefail
O=gpurun_out/f16; mkdir -p $O
for w in 2 3 8; do WAVES_PER_SIMD=$w timeout -k 10 120 ./scripts/ubench/f16_rate > $O/w$w.txt 2>&1 || exit 1; done
echo RC=0; cat $O/w*.txt
