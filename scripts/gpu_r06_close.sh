# Round 6 close on the final sources: smoke(), the default bench line as the
# driver runs it (with cpu_baseline and both parity legs), C3 and C5 lines,
# a kernel trace of the default bench command (rocprofv3 --kernel-trace
# --stats), into gpurun_out/$RUN; then (SHARES=1) every rank's share at N = 8.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06close}
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH FAILED; tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-300
for c in c3 c5; do
  timeout -k 10 900 python3 bench.py --config $c --no-cpu-baseline > $O/$c.json 2> $O/$c.err || { echo "$c FAILED"; tail -20 $O/$c.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$c.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$c', d['value'], d['ms_per_step'], r.get('value'), d.get('parity_sample_ok'), r.get('parity_ok'), d.get('cold_first_scan_ms'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-verify --steps 20 > $O/kt.json 2> $O/kt.err || { echo TRACE FAILED; tail -5 $O/kt.err; exit 1; }
cp $(find $O/kt -name "*kernel_stats.csv") $O/c2_kernel_stats.csv
head -6 $O/c2_kernel_stats.csv | cut -d, -f1-8 | cut -c1-160
if [ -n "$SHARES" ]; then RUN=$RUN/shares NS=${NS:-8} bash scripts/gpu_r06_shares.sh || exit 1; fi
echo RC=0
