# C5's workgroup rounds: 8 subjects per workgroup, 768 resident (3 per CU
# at RI 16), so 6,144 subjects fill one round; 10,000 = 1.63 rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/c5tail
mkdir -p $O
for n in 6144 10000 12288 20000; do
  timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --no-reference-scoring --db-seqs $n > $O/n$n.json 2> $O/n$n.err || exit $?
done
for n in 6144 10000 12288 20000; do python3 -c "
import json
d=json.loads(open('$O/n$n.json').read().strip().split(chr(10))[-1])
print($n, d['value'], d['kernels']['intra'], d['kernel_ms_per_scan']['sw_intra'])"; done
