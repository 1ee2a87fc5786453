# v10: column-biased fp16 cell (6 packed ops per cell pair): parity of the
# packed kernels, C2 bench (affine + reference scoring), C3 subset.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v24
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; echo RC=$rc; tail -3 $O/parity.log; cut -c1-1600 $O/bench.json; tail -3 $O/bench.err; exit $rc
