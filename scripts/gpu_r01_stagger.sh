# Staggered start of the intra workgroups (s_sleep by blockIdx % 3) vs none.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/stagger
mkdir -p $O
L=$PWD/ece1782-smith-waterman-cuda_amd
B="python3 bench.py --config c5 --no-cpu-baseline --no-reference-scoring"
for v in base st4 st32; do
  lib=""; [ $v != base ] && lib="SW_AMD_LIB=$L/lib_$v/libswamd.so"
  for n in 6144 10000; do
    env $lib timeout -k 10 300 $B --db-seqs $n > $O/${v}_$n.json 2> $O/${v}_$n.err || exit $?
  done
done
for v in base st4 st32; do for n in 6144 10000; do python3 -c "
import json
d=json.loads(open('$O/${v}_$n.json').read().strip().split(chr(10))[-1])
print('$v', $n, d['value'], d['kernel_ms_per_scan']['sw_intra'])"; done; done
