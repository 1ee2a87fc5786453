# Round 2: wave quads (G = 4) for small databases: parity, then the strong-
# scaling shares against group size, group width and the long threshold.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02d}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "wave_pair or saturation or guard_band" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
run() { tag=$1; shift; timeout -k 10 200 env "$@" python3 bench.py --no-reference-scoring --no-verify $BARGS > $O/$tag.json 2> $O/$tag.err || exit 1; }
BARGS="--shard-of 8 --long-threshold 704"
run s8_t704_g2 SW_PAIR_GROUP=2
run s8_t704_g4 SW_PAIR_GROUP=4
run s8_t704_g4_w16 SW_PAIR_GROUP=4 SW_PAIR_WIDTH=16
BARGS="--shard-of 8 --long-threshold 512"; run s8_t512_g4 SW_PAIR_GROUP=4
BARGS="--shard-of 8 --long-threshold 1024"; run s8_t1024_g4 SW_PAIR_GROUP=4
BARGS="--shard-of 4 --long-threshold 1024"; run s4_t1024_g4 SW_PAIR_GROUP=4
BARGS="--shard-of 4 --long-threshold 1536"; run s4_t1536_g4 SW_PAIR_GROUP=4
BARGS="--shard-of 2 --long-threshold 2048"; run s2_t2048_g4 SW_PAIR_GROUP=4
BARGS="--shard-of 2 --long-threshold 1536"; run s2_t1536_g4 SW_PAIR_GROUP=4
BARGS=""; run c2_g2 SW_PAIR_GROUP=2
BARGS=""; run c2_g4 SW_PAIR_GROUP=4
echo RC=0; tail -2 $O/tests.log
for f in $O/*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().split(chr(10))[-1])
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d.get('kernel_ms_per_scan'), d['config']['long_subjects_rank0'])"; done
