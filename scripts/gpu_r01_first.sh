set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/parity2.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke2.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench2.json 2> gpurun_out/bench2.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof2.log 2>&1
rc=$?
echo "RC=$rc"
tail -3 gpurun_out/parity2.log; cat gpurun_out/smoke2.log; cat gpurun_out/bench2.json; tail -5 gpurun_out/bench2.err
exit $rc
