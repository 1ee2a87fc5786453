# GPU tests + bench, then a 2-rank rehearsal of bench.py's multi-rank path on
# this single GPU (gloo collectives, both ranks on cuda:0).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/parity_d.log 2>&1 && \
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_d1.json 2> gpurun_out/bench_d1.err && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --backend gloo --device 0 --db-seqs 200000 > gpurun_out/bench_d2.json 2> gpurun_out/bench_d2.err
rc=$?; echo RC=$rc; tail -2 gpurun_out/parity_d.log; cat gpurun_out/bench_d1.json; cat gpurun_out/bench_d2.json; tail -5 gpurun_out/bench_d2.err; exit $rc
