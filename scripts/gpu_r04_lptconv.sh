# Round 4 A/B: the merged launch's intra forms (the long subjects' pairs and
# the pipelined longest pairs) with the LDS conveyor (default build) and
# without (lib/ab_lpt, X2FLAGS=-DSW_LPT_CONV=0), on C2's 1/8 share (both
# scorings in each line), C3 and C2, alternating, after the GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r04lptconv}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
b() { tag=$1; shift; timeout -k 10 600 python3 bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$tag', d['value'], d['ms_per_step'], d['kernels'], r.get('value'), d.get('parity_sample_ok'), (d.get('sustained') or {}).get('value'))"; }
AB=ece1782-smith-waterman-cuda_amd/lib/ab_lpt/libswamd.so
b s8_conv --shard-of 8
SW_AMD_LIB=$AB b s8_noconv --shard-of 8
b s8_convb --shard-of 8
SW_AMD_LIB=$AB b s8_noconvb --shard-of 8
b c3_conv --config c3
SW_AMD_LIB=$AB b c3_noconv --config c3
b c2_conv
SW_AMD_LIB=$AB b c2_noconv
echo RC=0
