# Round 2: the pipelined longest pairs again, ordered first (their estimate
# scaled), on C2's 1/8 share; block/workgroup timelines of the best case.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02m}
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 200 env "$@" python3 bench.py --no-reference-scoring --no-verify $BARGS > $O/$tag.json 2> $O/$tag.err || exit 1; }
BARGS="--shard-of 8"
run p0 SW_PIPE_LEN=0
run p3000_c1 SW_PIPE_LEN=3000
run p3000_c3 SW_PIPE_LEN=3000 SW_PIPE_COST=3
run p3000_c100 SW_PIPE_LEN=3000 SW_PIPE_COST=100
run p2000_c100 SW_PIPE_LEN=2000 SW_PIPE_COST=100
run p1500_c3 SW_PIPE_LEN=1500 SW_PIPE_COST=3
BARGS="--shard-of 8 --long-threshold 700"
run t700_p0 SW_PIPE_LEN=0
run t700_p2000_c100 SW_PIPE_LEN=2000 SW_PIPE_COST=100
L=ece1782-smith-waterman-cuda_amd/lib_trace/libswamd.so
SW_PIPE_LEN=3000 SW_PIPE_COST=100 SW_AMD_LIB=$L SW_TRACE_FILE=/tmp/tr.bin timeout -k 10 200 python3 scripts/exp_share_trace.py 8 0 > $O/trace_p3000_c100.json 2> $O/trace.err || exit 1
echo RC=0
for f in $O/p*.json $O/t*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().split(chr(10))[-1])
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d.get('kernel_ms_per_scan')['scan_total'], d['config']['long_threshold'])" 2>/dev/null; done; cat $O/trace_p3000_c100.json
