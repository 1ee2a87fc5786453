# Round 2 extras: C4 with all 50M subjects on one GPU, and a 4-rank torchrun
# rehearsal of the strong-scaled C2 (gloo, every rank on this one GPU) with
# the whole-database parity check.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02extra}
mkdir -p $O
timeout -k 10 600 python3 bench.py --config c4 --steps 3 --warmup 1 > $O/c4_full.json 2> $O/c4_full.err && \
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --backend gloo --device 0 --steps 20 > $O/c2_4rank_gloo.json 2> $O/c2_4rank_gloo.err
rc=$?; echo RC=$rc; for f in $O/*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d.get('reference_scoring') or {}; print('$f', d['value'], d['ms_per_step'], d['n_gpus'], '| ref', r.get('value'), '| parity', d.get('parity_sample_ok'), json.dumps(d.get('parity'))[:300])"; done; exit $rc
