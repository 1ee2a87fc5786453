# Inter kernels' guard-band early exit (default) vs none (lib_e0): GPU
# suite, C2, C3 (where long queries under the reference scoring flag blocks).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/early
mkdir -p $O
L=$PWD/ece1782-smith-waterman-cuda_amd
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/parity.log 2>&1 && \
B="python3 bench.py --no-cpu-baseline" && \
timeout -k 10 300 $B > $O/c2_e1.json 2> $O/c2_e1.err && \
SW_AMD_LIB=$L/lib_e0/libswamd.so timeout -k 10 300 $B > $O/c2_e0.json 2> $O/c2_e0.err && \
timeout -k 10 600 $B --config c3 > $O/c3_e1.json 2> $O/c3_e1.err && \
SW_AMD_LIB=$L/lib_e0/libswamd.so timeout -k 10 600 $B --config c3 > $O/c3_e0.json 2> $O/c3_e0.err
rc=$?; echo RC=$rc; tail -1 $O/parity.log
for f in c2_e1 c2_e0 c3_e1 c3_e0; do [ -f $O/$f.json ] && python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f', d['value'], d['kernel_ms_per_scan'], r.get('value'), r.get('kernel_ms_per_scan'))"; done; exit $rc
