# Chained-pass transitions staged by LDS-DMA a sub-group ahead (default) vs
# ordinary loads at the transition (lib_base): full GPU suite, then C2 / C3 A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/preload
mkdir -p $O
L=$PWD/ece1782-smith-waterman-cuda_amd
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/parity.log 2>&1 && \
B="python3 bench.py --no-cpu-baseline" && \
timeout -k 10 300 $B > $O/c2_c1.json 2> $O/c2_c1.err && \
SW_AMD_LIB=$L/lib_base/libswamd.so timeout -k 10 300 $B > $O/c2_c0.json 2> $O/c2_c0.err && \
timeout -k 10 300 $B > $O/c2_c1b.json 2> $O/c2_c1b.err && \
SW_AMD_LIB=$L/lib_base/libswamd.so timeout -k 10 300 $B > $O/c2_c0b.json 2> $O/c2_c0b.err && \
timeout -k 10 600 $B --config c3 > $O/c3_c1.json 2> $O/c3_c1.err && \
SW_AMD_LIB=$L/lib_base/libswamd.so timeout -k 10 600 $B --config c3 > $O/c3_c0.json 2> $O/c3_c0.err
rc=$?; echo RC=$rc; tail -3 $O/parity.log | cut -c1-300
for f in c2_c1 c2_c0 c2_c1b c2_c0b c3_c1 c3_c0; do [ -f $O/$f.json ] && python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f', d['value'], d['kernel_ms_per_scan']['sw_inter'], r.get('value'), r.get('kernel_ms_per_scan',{}).get('sw_inter'), d.get('parity_sample_ok'))"; done; exit $rc
