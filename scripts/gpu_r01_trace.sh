# Block timeline of the C2 scan (trace build) + default-build bench with the
# new pair width.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/trace
mkdir -p $O
SW_AMD_LIB=$PWD/ece1782-smith-waterman-cuda_amd/lib_trace/libswamd.so SW_TRACE_FILE=$PWD/$O/c2.trace timeout -k 10 300 python3 scripts/exp_tail_trace.py > $O/c2_trace.json 2> $O/c2_trace.err && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; echo RC=$rc; cat $O/c2_trace.json; tail -3 $O/c2_trace.err; python3 -c "
import json
d=json.loads(open('$O/bench.json').read().strip().split(chr(10))[-1]); print(d['value'], d['kernel_ms_per_scan'], d['reference_scoring']['value'])"; exit $rc
