# Round 5 close: smoke(), the default bench line exactly as the driver runs
# it (N = 1, cpu_baseline, parity), and a kernel trace of the default
# workload, into gpurun_out/$RUN.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r05close}
mkdir -p $O
timeout -k 10 600 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 900 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH FAILED; tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-verify --steps 20 > $O/kt.json 2> $O/kt.err || { echo TRACE FAILED; tail -5 $O/kt.err; exit 1; }
cp $(find $O/kt -name "*kernel_stats.csv") $O/c2_kernel_stats.csv
head -6 $O/c2_kernel_stats.csv | cut -d, -f1-8 | cut -c1-160
echo RC=0
