# Round 3 A/B: the GPU suite, then the intra work queue on/off (C5, C3) and
# the paired inter steps on/off (C2: lib vs lib_base built with -DSW_X2_PAIR=0)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-s3ql}; mkdir -p $O
LB=ece1782-smith-waterman-cuda_amd/lib_base/libswamd.so
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
run() { tag=$1; shift; env "$@" timeout -k 10 600 python3 bench.py --config $cfg > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$tag', d['value'], d['ms_per_step'], r.get('value'), d.get('parity_sample_ok'))"; }
# (c2 pair/base lines: lib built with the paired steps, lib_base with -DSW_X2_PAIR=0)
for cfg in c2; do for i in 1 2; do run ${cfg}_pair_$i X=1; run ${cfg}_base_$i SW_AMD_LIB=$LB; done; done
for cfg in c5 c3; do run ${cfg}_q1 SW_INTRA_QUEUE=1; run ${cfg}_q0 SW_INTRA_QUEUE=0; done
