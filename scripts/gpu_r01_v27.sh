# v27: full GPU suite, smoke, kernel-trace stats + PMC traffic of the C2
# command, the default bench line (CPU baseline included) reading that
# traffic, C3, C5, C4 (one rank's share of 8 GPUs).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-v27}
mkdir -p $O
KEY=P07327/570000/375/blosum62-12-1
B="python3 bench.py --no-cpu-baseline --no-reference-scoring --steps 3 --warmup 1"
sq() { name=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/$name -o run --output-format csv -- $B > $O/$name.json 2> $O/$name.err; }
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-reference-scoring --steps 10 --warmup 2 > $O/kt.json 2> $O/kt.err && \
sq fetch FETCH_SIZE && sq write WRITE_SIZE && \
python3 scripts/pmc_traffic.py $(dirname $(find $O/fetch -name run_counter_collection.csv)) $(dirname $(find $O/write -name run_counter_collection.csv)) $KEY $O/pmc_traffic.json "sw_inter_x2p<32, 8, true, true, true>" "sw_inter_x2p<32,8,affine,fp16>" > $O/traffic.log && \
timeout -k 10 600 python3 bench.py --traffic-json $O/pmc_traffic.json > $O/bench.json 2> $O/bench.err && \
timeout -k 10 600 python3 bench.py --config c5 > $O/c5.json 2> $O/c5.err && \
timeout -k 10 900 python3 bench.py --config c3 > $O/c3.json 2> $O/c3.err && \
timeout -k 10 600 python3 bench.py --config c4 --db-seqs 6250000 --steps 5 --warmup 1 > $O/c4_share8.json 2> $O/c4_share8.err
rc=$?; echo RC=$rc; tail -2 $O/parity.log; cat $O/smoke.log; cat $O/traffic.log | cut -c1-300; for f in bench c5 c3 c4_share8; do [ -f $O/$f.json ] && python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f', d['value'], d['ms_per_step'], d['dtype'], d['kernels'], r.get('value'), d.get('cpu_baseline',{}).get('value'), d.get('valu_roofline',{}).get('frac'), d['roofline'].get('traffic'))"; done; exit $rc
