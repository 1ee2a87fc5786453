# Round 3 A/B: the pair-image intra form (sw_intra_x2w, 12 waves per
# workgroup; lib_base: 8 waves) against sw_intra_x2 (SW_IX2_WIDE=0), after the
# GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-s3w}; mkdir -p $O
LB=ece1782-smith-waterman-cuda_amd/lib_base/libswamd.so
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
run() { tag=$1; shift; env "$@" timeout -k 10 600 python3 bench.py $ARGS > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$tag', d['value'], d['ms_per_step'], r.get('value'), d.get('parity_sample_ok'), d.get('kernels'))"; }
ARGS="--config c5"; run c5_w12 X=1; run c5_w8 SW_AMD_LIB=$LB; run c5_old SW_IX2_WIDE=0
ARGS="--config c3"; run c3_w12 X=1; run c3_old SW_IX2_WIDE=0
ARGS=""; run c2_w12 X=1; run c2_old SW_IX2_WIDE=0
ARGS="--shard-of 4"; run s4_w12 X=1; run s4_old SW_IX2_WIDE=0
