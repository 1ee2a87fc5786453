# Round 2: C5 at each rows-per-lane shape of the long-subject kernel
# (SW_INTRA_X2_RI), to check the shape model's choice (RI 16) against
# occupancy and the last round of workgroups.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02ae}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-verify --config c5 --steps 20 --warmup 2"
for ri in 16 12 10 8; do
  SW_INTRA_X2_RI=$ri timeout -k 10 300 $B > $O/c5_ri$ri.json 2> $O/c5_ri$ri.err || exit 1
done
for f in $O/*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d.get('reference_scoring') or {}; print('$f', d['value'], d['ms_per_step'], d['kernels'], '| ref', r.get('value'), r.get('ms_per_step'), r.get('intra_kernel'))"; done
