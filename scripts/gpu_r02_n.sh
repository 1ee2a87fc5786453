# Round 2: the whole C2 database with fewer long subjects (higher threshold,
# quads / merged launch) — is the concurrent long-subject kernel worth it?
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02n}
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 200 env "$@" python3 bench.py --no-reference-scoring --no-verify --no-cpu-baseline $BARGS > $O/$tag.json 2> $O/$tag.err || exit 1; }
BARGS=""; run def
BARGS=""; run serial SW_INTRA_SERIAL=1
BARGS="--long-threshold 3072"; run t3072
BARGS="--long-threshold 3072"; run t3072_lpt SW_LPT=1
BARGS="--long-threshold 4096"; run t4096_g4 SW_PAIR_GROUP=4
BARGS="--long-threshold 4096"; run t4096_lpt SW_LPT=1 SW_QUAD_WIDTH=2048
BARGS="--long-threshold 2048"; run t2048_lpt_q1400 SW_LPT=1 SW_QUAD_WIDTH=1400
echo RC=0
for f in $O/*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().split(chr(10))[-1])
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['kernels']['inter'], d.get('kernel_ms_per_scan'), d['config']['long_subjects_rank0'])" 2>/dev/null; done
