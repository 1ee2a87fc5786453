# Round 2: share-8 kernels alone (serial) to size the merged-launch idea.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02f}
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 200 env "$@" python3 bench.py --no-reference-scoring --no-verify $BARGS > $O/$tag.json 2> $O/$tag.err || exit 1; }
BARGS="--shard-of 8 --long-threshold 704"
run s8_t704_serial_g2 SW_INTRA_SERIAL=1 SW_PAIR_GROUP=2
run s8_t704_serial_g4 SW_INTRA_SERIAL=1 SW_PAIR_GROUP=4
run s8_t704_serial_g2_w64 SW_INTRA_SERIAL=1 SW_PAIR_GROUP=2 SW_PAIR_WIDTH=64
run s8_t704_serial_g4_w64 SW_INTRA_SERIAL=1 SW_PAIR_GROUP=4 SW_PAIR_WIDTH=64
BARGS="--shard-of 8 --long-threshold 1024"
run s8_t1024_serial_g4 SW_INTRA_SERIAL=1 SW_PAIR_GROUP=4
run s8_t1024_serial_g4_w64 SW_INTRA_SERIAL=1 SW_PAIR_GROUP=4 SW_PAIR_WIDTH=64
BARGS="--shard-of 8"
run s8_default
BARGS="--shard-of 4"
run s4_default
BARGS="--shard-of 2"
run s2_default
echo RC=0
for f in $O/*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().split(chr(10))[-1])
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d.get('kernel_ms_per_scan'), d['config']['long_subjects_rank0'], d['config']['long_threshold'])"; done
