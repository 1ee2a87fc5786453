# Round 5 iteration check: the GPU suite (or only tests matching $FIRST
# first), then the configs in $CONFIGS (default: C2 and its 1/8 share), and
# with TRACE=1 a rocprofv3 kernel trace of the 1/8 share (per-dispatch start /
# end: the launches around the merged scan, scripts/step_gaps.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r05quick}
mkdir -p $O
if [ -n "$FIRST" ]; then timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "$FIRST" --timeout 200 --timeout-method thread > $O/first_tests.log 2>&1 || { echo FIRST TESTS FAILED; tail -40 $O/first_tests.log; exit 1; }; tail -1 $O/first_tests.log; fi
if [ -z "$NOSUITE" ]; then timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/gpu_tests.log; exit 1; }; tail -1 $O/gpu_tests.log; fi
b() { tag=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -20 $O/$tag.err; exit 1; }; }
for c in ${CONFIGS:-c2 s8}; do
  case $c in
    c2) b c2 --no-cpu-baseline ;;
    s8) b s8 --shard-of 8 --no-cpu-baseline ;;
    s4) b s4 --shard-of 4 --no-cpu-baseline ;;
    s2) b s2 --shard-of 2 --no-cpu-baseline ;;
    c3) b c3 --config c3 --no-cpu-baseline ;;
    c5) b c5 --config c5 --no-cpu-baseline ;;
  esac
  python3 -c "
import json
d=json.loads(open('$O/$c.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$c', d['value'], d['ms_per_step'], d.get('kernel_ms_per_scan',{}).get('scan_total'), r.get('value'), r.get('ms_per_step'), d.get('parity_sample_ok'), d.get('sustained',{}).get('value') if d.get('sustained') else None)"
done
# TRACE="c2 s8": rocprofv3 kernel traces (per-kernel stats) of those configs
for c in $TRACE; do
  case $c in c2) a="" ;; s8) a="--shard-of 8" ;; s4) a="--shard-of 4" ;; c5) a="--config c5" ;; c3) a="--config c3 --steps 3 --warmup 1" ;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$c -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-verify --no-reference-scoring $a > $O/kt_$c.json 2> $O/kt_$c.err || { echo TRACE $c FAILED; tail -5 $O/kt_$c.err; exit 1; }
  head -8 $(find $O/kt_$c -name "*kernel_stats.csv") | cut -d, -f1-8 | cut -c1-150
done
echo RC=0
