# Round 2: the drop-in C++ path at Swiss-Prot scale + group API tests +
# long-threshold sweeps of the strong-scaling shares.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02c}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_cli.py tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 900 python3 -u scripts/dropin_scale.py --n 570000 --gpus2 --out /tmp/dropin > $O/dropin_570k.json 2> $O/dropin_570k.err && \
for s in 2 4; do for t in 1024 1536 2048; do
  timeout -k 10 200 python3 bench.py --shard-of $s --no-reference-scoring --no-verify --long-threshold $t > $O/s${s}_t$t.json 2> $O/s${s}_t$t.err || exit 1
done; done && \
for t in 600 800; do
  timeout -k 10 200 python3 bench.py --shard-of 8 --no-reference-scoring --no-verify --long-threshold $t > $O/s8_t$t.json 2> $O/s8_t$t.err || exit 1
done
rc=$?; echo RC=$rc; tail -3 $O/tests.log; cat $O/dropin_570k.json | cut -c1-3000
for f in $O/s*_t*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().split(chr(10))[-1])
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d.get('kernel_ms_per_scan'), d['config']['long_subjects_rank0'])"; done; exit $rc
