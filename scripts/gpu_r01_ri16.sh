# C5 (affine + reference scoring) with the intra rows per lane forced.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ri16
mkdir -p $O
for ri in 8 10 12 16; do
  SW_INTRA_X2_RI=$ri timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline > $O/ri$ri.json 2> $O/ri$ri.err || exit $?
done
for ri in 8 10 12 16; do python3 -c "
import json
d=json.loads(open('$O/ri$ri.json').read().strip().split(chr(10))[-1]); r=d['reference_scoring']
print($ri, d['value'], r['value'], r['intra_kernel'])"; done
