# Parity, kernel-trace stats of the bench command, two PMC passes for the
# dominant kernel's HBM bytes, then the bench line that reads them.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-traffic}
mkdir -p $O
KEY=P07327/570000/375/blosum62-12-1
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/parity.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-verify --no-reference-scoring --steps 10 --warmup 2 > $O/kt.json 2> $O/kt.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-verify --no-reference-scoring --steps 3 --warmup 1 > $O/fetch.json 2> $O/fetch.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-verify --no-reference-scoring --steps 3 --warmup 1 > $O/write.json 2> $O/write.err && \
python3 scripts/pmc_traffic.py $(dirname $(find $O/fetch -name run_counter_collection.csv)) $(dirname $(find $O/write -name run_counter_collection.csv)) $KEY $O/pmc_traffic.json "sw_inter_x2p<32, 8, true, true, true, 2>" "sw_inter_x2p<32,8,affine,fp16>" > $O/traffic.log && \
timeout -k 10 900 python3 bench.py --traffic-json $O/pmc_traffic.json > $O/bench.json 2> $O/bench.err
rc=$?; echo RC=$rc; tail -2 $O/parity.log; cat $O/traffic.log; cat $O/bench.json; tail -3 $O/bench.err; exit $rc
