# Radix-select top-K: its tests, then C2 under rocprofv3 kernel-trace stats.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/topk
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k topk --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; echo RC=$rc; tail -3 $O/tests.log
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && python3 -c "
import csv
for r in csv.DictReader(open('$f')): print(r['Name'][:60], r['Calls'], r['AverageNs'])"
exit $rc
