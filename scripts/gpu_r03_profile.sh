# Round 3 profiles of the default bench (C2, N = 1): kernel-trace stats, two
# PMC passes for the dominant kernel's HBM bytes, one SQ pass for its VALU
# instructions, the stored measurement folded into pmc_traffic.json, then
# the bench line that reads it; kernel-trace stats of the 1/8 share too.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r03prof}
mkdir -p $O
KEY=P07327/570000/375/blosum62-12-1
B="bench.py --no-cpu-baseline --no-verify --no-reference-scoring"
K="sw_inter_x2p<32, 8, true, true, true, 2>"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $B --steps 20 --warmup 2 > $O/kt.json 2> $O/kt.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_s8 -o run --output-format csv -- python3 $B --shard-of 8 --steps 50 --warmup 2 > $O/kt_s8.json 2> $O/kt_s8.err && \
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $B --steps 3 --warmup 1 > $O/fetch.json 2> $O/fetch.err && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $B --steps 3 --warmup 1 > $O/write.json 2> $O/write.err && \
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $O/sq -o run --output-format csv -- python3 $B --steps 3 --warmup 1 > $O/sq.json 2> $O/sq.err && \
python3 scripts/pmc_traffic.py $(dirname $(find $O/fetch -name run_counter_collection.csv)) $(dirname $(find $O/write -name run_counter_collection.csv)) $KEY $O/pmc_traffic.json "$K" "sw_inter_x2p<32,8,affine,fp16>" $(dirname $(find $O/sq -name run_counter_collection.csv)) > $O/traffic.log && \
python3 scripts/pmc_summary.py $(dirname $(find $O/sq -name run_counter_collection.csv)) > $O/sq_summary.txt && \
timeout -k 10 600 python3 bench.py --traffic-json $O/pmc_traffic.json > $O/bench.json 2> $O/bench.err
rc=$?; echo RC=$rc; cat $O/traffic.log; head -5 $(find $O/kt -name "*kernel_stats.csv") | cut -c1-200; head -6 $(find $O/kt_s8 -name "*kernel_stats.csv") | cut -c1-200; cat $O/bench.json | cut -c1-1500; exit $rc
