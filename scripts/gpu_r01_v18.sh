# v18 (row+column biased fp16 cells, affine and linear): full GPU
# stats of the bench command, PMC traffic (FETCH/WRITE) and SQ counters of the
# dominant kernel, then the default bench line that reads the traffic, C3, C5.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v18
mkdir -p $O
KEY=P07327/570000/375/blosum62-12-1
B="python3 bench.py --no-cpu-baseline --no-reference-scoring --steps 3 --warmup 1"
sq() { name=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/$name -o run --output-format csv -- $B > $O/$name.json 2> $O/$name.err; }
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-reference-scoring --steps 10 --warmup 2 > $O/kt.json 2> $O/kt.err && \
sq fetch FETCH_SIZE && sq write WRITE_SIZE && \
sq sqa SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE && \
sq sqb SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS && \
python3 scripts/pmc_traffic.py $(dirname $(find $O/fetch -name run_counter_collection.csv)) $(dirname $(find $O/write -name run_counter_collection.csv)) $KEY $O/r01_pmc_traffic.json "sw_inter_x2p<32, 8, true, true, true>" "sw_inter_x2p<32,8,affine,fp16>" > $O/traffic.log && \
python3 scripts/pmc_summary.py $(dirname $(find $O/sqa -name run_counter_collection.csv)) $(dirname $(find $O/sqb -name run_counter_collection.csv)) > $O/sq_summary.txt && \
timeout -k 10 600 python3 bench.py --traffic-json $O/r01_pmc_traffic.json > $O/bench.json 2> $O/bench.err && \
timeout -k 10 600 python3 bench.py --config c5 > $O/c5.json 2> $O/c5.err && \
timeout -k 10 900 python3 bench.py --config c3 > $O/c3.json 2> $O/c3.err
rc=$?; echo RC=$rc; tail -2 $O/parity.log; cat $O/traffic.log; for f in bench c5 c3; do echo "== $f"; cut -c1-600 $O/$f.json; tail -2 $O/$f.err; done; exit $rc
