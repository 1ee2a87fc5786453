# Intra kernel with the next step's LDS words prefetched (default) vs not
# (lib_p0): intra parity, C5 at 10,000 and 6,144 subjects, C2.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prefetch
mkdir -p $O
L=$PWD/ece1782-smith-waterman-cuda_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "intra or golden or synthetic" --timeout 120 --timeout-method thread > $O/parity.log 2>&1 && \
B="python3 bench.py --no-cpu-baseline" && \
timeout -k 10 300 $B --config c5 > $O/c5_p1.json 2> $O/c5_p1.err && \
SW_AMD_LIB=$L/lib_p0/libswamd.so timeout -k 10 300 $B --config c5 > $O/c5_p0.json 2> $O/c5_p0.err && \
timeout -k 10 300 $B --config c5 --db-seqs 6144 --no-reference-scoring > $O/c5s_p1.json 2> $O/c5s_p1.err && \
SW_AMD_LIB=$L/lib_p0/libswamd.so timeout -k 10 300 $B --config c5 --db-seqs 6144 --no-reference-scoring > $O/c5s_p0.json 2> $O/c5s_p0.err && \
timeout -k 10 300 $B > $O/c2_p1.json 2> $O/c2_p1.err && \
SW_AMD_LIB=$L/lib_p0/libswamd.so timeout -k 10 300 $B > $O/c2_p0.json 2> $O/c2_p0.err
rc=$?; echo RC=$rc; tail -1 $O/parity.log
for f in c5_p1 c5_p0 c5s_p1 c5s_p0 c2_p1 c2_p0; do [ -f $O/$f.json ] && python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f', d['value'], d['kernels']['intra'], d['kernel_ms_per_scan']['sw_intra'], r.get('value'), r.get('kernel_ms_per_scan',{}).get('sw_intra'))"; done; exit $rc
