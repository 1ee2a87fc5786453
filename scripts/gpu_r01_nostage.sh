# Timing-only: chained passes without the transition work (wrong scores) vs default.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/nostage
mkdir -p $O
L=$PWD/ece1782-smith-waterman-cuda_amd
B="python3 bench.py --no-cpu-baseline --no-reference-scoring"
timeout -k 10 300 $B > $O/d1.json 2> $O/d1.err && \
SW_AMD_LIB=$L/lib_ns/libswamd.so timeout -k 10 300 $B > $O/n1.json 2> $O/n1.err && \
timeout -k 10 300 $B > $O/d2.json 2> $O/d2.err && \
SW_AMD_LIB=$L/lib_ns/libswamd.so timeout -k 10 300 $B > $O/n2.json 2> $O/n2.err
rc=$?; echo RC=$rc
for f in d1 n1 d2 n2; do [ -f $O/$f.json ] && python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); print('$f', d['value'], d['kernel_ms_per_scan']['sw_inter'])"; done; exit $rc
