# Round 5 closing run on the round's last kernels: the whole GPU suite,
# smoke(), the default bench line as the driver runs it (N = 1,
# cpu_baseline, parity), a kernel trace of the default workload, then the
# bench lines (parity on, both scorings) of C3, C5 and C2's 1/2, 1/4 and
# 1/8 shares, into gpurun_out/$RUN.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r05final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
RUN=${RUN:-r05final} bash scripts/gpu_r05_close.sh || exit 1
for c in c3 c5 s2 s4 s8; do
  case $c in c3) a="--config c3" ;; c5) a="--config c5" ;; s2) a="--shard-of 2" ;; s4) a="--shard-of 4" ;; s8) a="--shard-of 8" ;; esac
  timeout -k 10 600 python3 bench.py $a --no-cpu-baseline --sustained-seconds 0 > $O/$c.json 2> $O/$c.err || { echo "BENCH $c FAILED"; tail -5 $O/$c.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); r=d.get('reference_scoring') or {}
print(sys.argv[2], d['value'], d['ms_per_step'], r.get('value'), d['roofline']['kernel'])" $O/$c.json $c
done
echo RC=0
