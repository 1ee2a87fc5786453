# v20: full GPU suite, kernel-trace stats + PMC traffic of the C2 command, the
# default bench line (CPU baseline included), C3, C5, C4 (one rank's share of
# 8 GPUs, and all 50M subjects on one GPU).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v20
mkdir -p $O
KEY=P07327/570000/375/blosum62-12-1
B="python3 bench.py --no-cpu-baseline --no-reference-scoring --steps 3 --warmup 1"
sq() { name=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/$name -o run --output-format csv -- $B > $O/$name.json 2> $O/$name.err; }
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-reference-scoring --steps 10 --warmup 2 > $O/kt.json 2> $O/kt.err && \
sq fetch FETCH_SIZE && sq write WRITE_SIZE && \
python3 scripts/pmc_traffic.py $(dirname $(find $O/fetch -name run_counter_collection.csv)) $(dirname $(find $O/write -name run_counter_collection.csv)) $KEY $O/r01_pmc_traffic.json "sw_inter_x2p<32, 8, true, true, true>" "sw_inter_x2p<32,8,affine,fp16>" > $O/traffic.log && \
timeout -k 10 600 python3 bench.py --traffic-json $O/r01_pmc_traffic.json > $O/bench.json 2> $O/bench.err && \
timeout -k 10 600 python3 bench.py --config c5 > $O/c5.json 2> $O/c5.err && \
timeout -k 10 900 python3 bench.py --config c3 > $O/c3.json 2> $O/c3.err && \
timeout -k 10 600 python3 bench.py --config c4 --db-seqs 6250000 --steps 5 --warmup 1 > $O/c4_share8.json 2> $O/c4_share8.err && \
timeout -k 10 900 python3 bench.py --config c4 --steps 3 --warmup 1 --no-reference-scoring > $O/c4_full.json 2> $O/c4_full.err
rc=$?; echo RC=$rc; tail -2 $O/parity.log; cat $O/traffic.log | cut -c1-300; for f in bench c5 c3 c4_share8 c4_full; do python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f', d['value'], d['ms_per_step'], d['dtype'], d['kernels'], r.get('value'), d.get('cpu_baseline',{}).get('value'), d.get('valu_roofline',{}).get('frac'))"; done; exit $rc
