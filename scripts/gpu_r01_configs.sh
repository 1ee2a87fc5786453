# Parity (incl. the C3 batch test), then bench lines for C2 (headline), C3, C5
# and a 2-rank gloo rehearsal of the multi-rank path.
set -o pipefail
O=gpurun_out/configs; mkdir -p $O
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/parity.log 2>&1 && \
timeout -k 10 600 python3 bench.py > $O/c2.json 2> $O/c2.err && \
timeout -k 10 900 python3 bench.py --config c3 > $O/c3.json 2> $O/c3.err && \
timeout -k 10 600 python3 bench.py --config c5 > $O/c5.json 2> $O/c5.err && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --backend gloo --device 0 --db-seqs 200000 --no-reference-scoring > $O/c2_2rank.json 2> $O/c2_2rank.err
rc=$?; echo RC=$rc; tail -2 $O/parity.log; for f in c2 c3 c5 c2_2rank; do echo "== $f"; cut -c1-1500 $O/$f.json; tail -2 $O/$f.err; done; exit $rc
