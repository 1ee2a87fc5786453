# Round 3 iteration check: the GPU suite, then C2, its 1/8 share and C3.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r03quick}
mkdir -p $O
if [ -n "$FIRST" ]; then timeout -k 10 240 python -u -m pytest tests -x -q -m gpu -k "$FIRST" --timeout 120 --timeout-method thread > $O/first_tests.log 2>&1 || { echo FIRST TESTS FAILED; tail -40 $O/first_tests.log; exit 1; }; tail -1 $O/first_tests.log; fi
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
b() { tag=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -20 $O/$tag.err; exit 1; }; }
for c in ${CONFIGS:-c2 s8 c3}; do
  case $c in
    c2) b c2 --no-cpu-baseline ;;
    s8) b s8 --shard-of 8 --no-cpu-baseline ;;
    s4) b s4 --shard-of 4 --no-cpu-baseline ;;
    c3) b c3 --config c3 --no-cpu-baseline ;;
    c5) b c5 --config c5 --no-cpu-baseline ;;
  esac
  python3 -c "
import json
d=json.loads(open('$O/$c.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$c', d['value'], d['ms_per_step'], d.get('kernel_ms_per_scan',{}).get('scan_total'), r.get('value'), r.get('ms_per_step'), d.get('parity_sample_ok'))"
done
