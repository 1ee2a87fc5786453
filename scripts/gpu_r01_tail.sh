# C2 tail experiments: wave-pair width, database size, long threshold.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/tail2
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-reference-scoring"
run() { name=$1; shift; timeout -k 10 300 env "$@" $B > $O/$name.json 2> $O/$name.err || return 1; }
run default X=1 && run nopair SW_PAIR_WIDTH=0 && run pair1024 SW_PAIR_WIDTH=1024 && run pair256 SW_PAIR_WIDTH=256 && \
timeout -k 10 300 $B --db-seqs 2280000 > $O/db4x.json 2> $O/db4x.err && \
timeout -k 10 300 $B --long-threshold 4096 > $O/lt4096.json 2> $O/lt4096.err && \
timeout -k 10 300 $B --long-threshold 1536 > $O/lt1536.json 2> $O/lt1536.err
rc=$?; echo RC=$rc; for f in default nopair pair1024 pair256 db4x lt4096 lt1536; do python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1])
print('$f', d['value'], d['ms_per_step'], d['kernel_ms_per_scan'], d['config']['long_subjects'], d['valu_roofline']['frac'])"; done; exit $rc
