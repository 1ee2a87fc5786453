# C5 routing: all-intra vs inter (+coop) for 5000-aa x 2000-aa subjects.
set -o pipefail
O=gpurun_out/c5; mkdir -p $O
B="bench.py --config c5 --no-cpu-baseline --no-reference-scoring --steps 3 --warmup 1"
timeout -k 10 300 python3 $B --long-threshold 1 > $O/intra.json 2> $O/intra.err && \
SW_COOP_WIDTH=128 timeout -k 10 300 python3 $B > $O/coop.json 2> $O/coop.err && \
SW_COOP_WIDTH=128 SW_INT16_GUARD=0 timeout -k 10 300 python3 $B > $O/coop32.json 2> $O/coop32.err && \
timeout -k 10 300 python3 $B --matrix blosum50 --gap-open 2 --gap-extend 2 --long-threshold 1 > $O/intra_lin.json 2> $O/intra_lin.err
rc=$?; echo RC=$rc; for f in intra coop coop32 intra_lin; do python3 -c "
import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms_per_scan'], d['roofline']['kernel'])"; done; exit $rc
