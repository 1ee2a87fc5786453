# v23: char-compat scoring (f4) tests, full GPU suite, 2-rank gloo rehearsal
# of bench.py's multi-rank path on this one GPU.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v23
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --backend gloo --device 0 --db-seqs 200000 --no-cpu-baseline > $O/bench_2rank.json 2> $O/bench_2rank.err
rc=$?; echo RC=$rc; tail -3 $O/parity.log; cut -c1-700 $O/bench_2rank.json; tail -3 $O/bench_2rank.err; exit $rc
