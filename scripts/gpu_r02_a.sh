# Round 2: strong-scaling bench, per-rank shares on one GPU, 2-rank gloo
# rehearsal, C1, and the new distributed GPU tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02a}
mkdir -p $O
(nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>&1) > $O/host.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread > $O/dist_tests.log 2>&1 && \
timeout -k 10 600 python3 bench.py > $O/c2.json 2> $O/c2.err && \
for s in 2 4 8; do timeout -k 10 300 python3 bench.py --shard-of $s --no-reference-scoring > $O/c2_share$s.json 2> $O/c2_share$s.err || exit 1; done && \
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --device 0 --steps 20 > $O/c2_2rank_gloo.json 2> $O/c2_2rank_gloo.err && \
timeout -k 10 300 python3 bench.py --config c1 > $O/c1.json 2> $O/c1.err
rc=$?; echo RC=$rc; cat $O/host.txt; tail -3 $O/dist_tests.log
for f in c2 c2_share2 c2_share4 c2_share8 c2_2rank_gloo c1; do [ -f $O/$f.json ] && python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f', d['value'], d['ms_per_step'], d.get('kernel_ms_per_scan'), r.get('value'), d.get('cpu_baseline',{}).get('value'), d.get('cpu_baseline',{}).get('one_thread'), d.get('parity_sample_ok'), d.get('parity'))"; done; exit $rc
