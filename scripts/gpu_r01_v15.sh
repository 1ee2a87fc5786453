# v15: b64 conflict-free LDS image reads (inline asm, manual waits) vs the
# b128 build (lib_b128): parity on b64, LDS-conflict experiment and C2 bench
# on both.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v15
mkdir -p $O
B128=$PWD/ece1782-smith-waterman-cuda_amd/lib_b128/libswamd.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 300 python3 scripts/exp_lds_conflict.py > $O/exp_b64.json 2> $O/exp_b64.err && \
SW_AMD_LIB=$B128 timeout -k 10 300 python3 scripts/exp_lds_conflict.py > $O/exp_b128.json 2> $O/exp_b128.err && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_b64.json 2> $O/bench_b64.err && \
SW_AMD_LIB=$B128 timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_b128.json 2> $O/bench_b128.err
rc=$?; echo RC=$rc; tail -3 $O/parity.log; cat $O/exp_b64.json $O/exp_b128.json; for f in b64 b128; do python3 -c "
import json,sys
d=json.loads(open('$O/bench_$f.json').read().strip().split(chr(10))[-1]); r=d['reference_scoring']
print('$f', d['value'], d['kernel_ms_per_scan']['sw_inter'], r['value'], r['kernel_ms_per_scan']['sw_inter'])"; done; exit $rc
