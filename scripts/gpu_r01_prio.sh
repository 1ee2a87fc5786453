# s_setprio 2 in the scan kernel (lib_pr2) vs default, C2 twice each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prio
mkdir -p $O
L=$PWD/ece1782-smith-waterman-cuda_amd
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 300 $B > $O/d1.json 2> $O/d1.err && \
SW_AMD_LIB=$L/lib_pr2/libswamd.so timeout -k 10 300 $B > $O/p1.json 2> $O/p1.err && \
timeout -k 10 300 $B > $O/d2.json 2> $O/d2.err && \
SW_AMD_LIB=$L/lib_pr2/libswamd.so timeout -k 10 300 $B > $O/p2.json 2> $O/p2.err
rc=$?; echo RC=$rc
for f in d1 p1 d2 p2; do [ -f $O/$f.json ] && python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f', d['value'], d['kernel_ms_per_scan'], r.get('value'), r.get('kernel_ms_per_scan'))"; done; exit $rc
