# v8 (wave-pair kernel for wide blocks, packed two-subjects intra kernel):
# parity, kernel-trace stats of the bench command, two PMC passes for the
# dominant kernel's HBM bytes, the C2 bench line that reads them, C5 and C3.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v8c
mkdir -p $O
KEY=P07327/570000/375/blosum62-12-1
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/parity.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-reference-scoring --steps 10 --warmup 2 > $O/kt.json 2> $O/kt.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-reference-scoring --steps 3 --warmup 1 > $O/fetch.json 2> $O/fetch.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-reference-scoring --steps 3 --warmup 1 > $O/write.json 2> $O/write.err && \
python3 scripts/pmc_traffic.py $(dirname $(find $O/fetch -name run_counter_collection.csv)) $(dirname $(find $O/write -name run_counter_collection.csv)) $KEY $O/r01_pmc_traffic.json "sw_inter_x2p<32, 8, true, true, true>" "sw_inter_x2p<32,8,affine,fp16>" > $O/traffic.log && \
timeout -k 10 900 python3 bench.py --traffic-json $O/r01_pmc_traffic.json > $O/bench.json 2> $O/bench.err && \
timeout -k 10 600 python3 bench.py --config c5 > $O/c5.json 2> $O/c5.err && \
timeout -k 10 900 python3 bench.py --config c3 > $O/c3.json 2> $O/c3.err
rc=$?; echo RC=$rc; tail -2 $O/parity.log; cat $O/traffic.log; for f in bench c5 c3; do echo "== $f"; cut -c1-900 $O/$f.json; tail -2 $O/$f.err; done; exit $rc
