# Round 2: wave priority for the merged launch's critical workgroups, and a
# 4-rank torchrun rehearsal (gloo, all ranks on this GPU) of the strong-
# scaling bench with its parity leg.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02l}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "lpt" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
run() { tag=$1; shift; timeout -k 10 200 env "$@" python3 bench.py --no-reference-scoring --no-verify $BARGS > $O/$tag.json 2> $O/$tag.err || exit 1; }
BARGS="--shard-of 8"
run s8_prio0 SW_LPT_PRIO=0
run s8_prio5 SW_LPT_PRIO=0.5
run s8_prio7 SW_LPT_PRIO=0.7
run s8_prio85 SW_LPT_PRIO=0.85
run s8_prio3 SW_LPT_PRIO=0.3
BARGS="--shard-of 4"
run s4_prio0 SW_LPT_PRIO=0
run s4_prio7 SW_LPT_PRIO=0.7
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --backend gloo --device 0 --steps 20 --no-reference-scoring > $O/c2_4rank_gloo.json 2> $O/c2_4rank_gloo.err || { echo RANK4 FAILED; tail -20 $O/c2_4rank_gloo.err; exit 1; }
echo RC=0; tail -2 $O/tests.log
for f in $O/*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().split(chr(10))[-1])
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d.get('kernel_ms_per_scan')['scan_total'], d['config']['long_threshold'], d.get('parity_sample_ok'), d.get('parity'))"; done
