# Round 6 close, part 2 (final sources): C1 and C4's ranks 0 and 7
# (scripts/gpu_r06_c14.sh), every rank's share at N = 2 and 4, and the
# multi-rank bench path end to end on the one GPU: `bench.py --gpus 2`
# launching its own torchrun ranks, gloo exchange, both ranks on device 0.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06close2}
mkdir -p $O
RUN=${RUN:-r06close2}/c14 bash scripts/gpu_r06_c14.sh || exit 1
RUN=${RUN:-r06close2}/shares NS="2 4" bash scripts/gpu_r06_shares.sh || exit 1
timeout -k 10 600 python3 bench.py --gpus 2 --backend gloo --device 0 --steps 20 --warmup 5 --no-cpu-baseline --sustained-seconds 0 > $O/gpus2_gloo.json 2> $O/gpus2_gloo.err || { echo GLOO2 FAILED; tail -20 $O/gpus2_gloo.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/gpus2_gloo.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('gpus2 gloo', d['n_gpus'], d['value'], d['ms_per_step'], d.get('parity_sample_ok'), d['parity']['merged_topk_equal'], r.get('parity_ok'))"
echo RC=0
