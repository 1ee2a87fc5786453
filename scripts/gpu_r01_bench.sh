# parity + smoke + bench + rocprof kernel-trace stats (one GPU call)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-x}
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/parity_$TAG.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?
echo "RC=$rc"
tail -3 gpurun_out/parity_$TAG.log; cat gpurun_out/smoke_$TAG.log; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
head -4 gpurun_out/prof_$TAG/run_kernel_stats.csv 2>/dev/null | cut -c1-200
exit $rc
