# Round 2: pipelined longest pairs in the merged launch — parity, then the
# shares against the pipe length.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02j}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "lpt or intra" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
run() { tag=$1; shift; timeout -k 10 200 env "$@" python3 bench.py --no-reference-scoring --no-verify $BARGS > $O/$tag.json 2> $O/$tag.err || exit 1; }
BARGS="--shard-of 8"
run s8_p0 SW_PIPE_LEN=0
run s8_pdef
run s8_p1200 SW_PIPE_LEN=1200
run s8_p2500 SW_PIPE_LEN=2500
run s8_p4000 SW_PIPE_LEN=4000
BARGS="--shard-of 8 --long-threshold 1200"; run s8_t1200_pdef
BARGS="--shard-of 8 --long-threshold 1500"; run s8_t1500_pdef
BARGS="--shard-of 4"
run s4_p0 SW_PIPE_LEN=0
run s4_pdef
BARGS="--shard-of 4 --long-threshold 1500"; run s4_t1500_pdef
echo RC=0; tail -2 $O/tests.log
for f in $O/*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().split(chr(10))[-1])
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d.get('kernel_ms_per_scan')['scan_total'], d['config']['long_subjects_rank0'], d['config']['long_threshold'])"; done
