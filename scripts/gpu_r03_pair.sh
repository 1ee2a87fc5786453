# Round 3 A/B: paired inter steps (lib) vs unpaired (lib_base, -DSW_X2_PAIR=0)
# on C2's strong-scaling shares, where few waves per SIMD leave dependency
# stalls unhidden
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-s3qm}; mkdir -p $O
LB=ece1782-smith-waterman-cuda_amd/lib_base/libswamd.so
run() { tag=$1; shift; env "$@" timeout -k 10 600 python3 bench.py $ARGS > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().split(chr(10))[-1])
print('$tag', d['value'], d['ms_per_step'], d.get('parity_sample_ok'))"; }
for n in 8 4 2; do ARGS="--shard-of $n"; for i in 1 2; do run s${n}_pair_$i X=1; run s${n}_base_$i SW_AMD_LIB=$LB; done; done
