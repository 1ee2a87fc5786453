# Round 2: the top-K exchange overlapped with the next scan (bench.py), one
# GPU and a 2-rank gloo rehearsal, against --no-overlap.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02o}
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -5 $O/$tag.err; exit 1; }; }
run c2_ovl --no-cpu-baseline
run c2_serial --no-cpu-baseline --no-overlap
run s8_ovl --shard-of 8
run s8_serial --shard-of 8 --no-overlap
run s4_ovl --shard-of 4 --no-reference-scoring
run c3_ovl --config c3 --no-cpu-baseline --no-reference-scoring
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29537 bench.py --gpus 2 --backend gloo --device 0 --steps 20 --no-reference-scoring > $O/r2_ovl.json 2> $O/r2_ovl.err || { echo RANK2 FAILED; tail -20 $O/r2_ovl.err; exit 1; }
echo RC=0
for f in $O/*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d.get('kernel_ms_per_scan')['scan_total'], r.get('value'), d.get('parity_sample_ok'), (d.get('parity') or {}).get('merged_topk_equal'), d['top_hit'])" 2>/dev/null; done
