# Round 4 profiles of the default bench (C2, N = 1; affine C2 runs the merged
# launch sw_scan_lpt): kernel-trace stats of C2, of its reference scoring and
# of the 1/8 share; two PMC passes per scoring for the dominant kernel's HBM
# bytes, one SQ pass for its VALU instructions; the affine measurement folded
# into pmc_traffic.json (the reference scoring's beside it), then the bench
# line that reads it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r04prof}
mkdir -p $O
KEY=P07327/570000/375/blosum62-12-1
KEYR=P07327/570000/375/blosum50-2-2
B="bench.py --no-cpu-baseline --no-verify --no-reference-scoring --sustained-seconds 0"
BR="$B --matrix blosum50 --gap-open 2 --gap-extend 2"
K="sw_scan_lpt<32, 8, true"
KR="sw_inter_x2p<32, 8, false"
csvdir() { dirname $(find $1 -name run_counter_collection.csv); }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $B --steps 20 --warmup 2 > $O/kt.json 2> $O/kt.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_ref -o run --output-format csv -- python3 $BR --steps 20 --warmup 2 > $O/kt_ref.json 2> $O/kt_ref.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_s8 -o run --output-format csv -- python3 $B --shard-of 8 --steps 50 --warmup 2 > $O/kt_s8.json 2> $O/kt_s8.err && \
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $B --steps 3 --warmup 1 > $O/fetch.json 2> $O/fetch.err && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $B --steps 3 --warmup 1 > $O/write.json 2> $O/write.err && \
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $O/sq -o run --output-format csv -- python3 $B --steps 3 --warmup 1 > $O/sq.json 2> $O/sq.err && \
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_ref -o run --output-format csv -- python3 $BR --steps 3 --warmup 1 > $O/fetch_ref.json 2> $O/fetch_ref.err && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/write_ref -o run --output-format csv -- python3 $BR --steps 3 --warmup 1 > $O/write_ref.json 2> $O/write_ref.err && \
python3 scripts/pmc_traffic.py $(csvdir $O/fetch) $(csvdir $O/write) $KEY $O/pmc_traffic.json "$K" "sw_inter_x2p<32,8,affine,fp16>+lpt+drain" $(csvdir $O/sq) > $O/traffic.log && \
python3 scripts/pmc_traffic.py $(csvdir $O/fetch_ref) $(csvdir $O/write_ref) $KEYR $O/pmc_traffic_ref.json "$KR" "sw_inter_x2p<32,8,linear,fp16>" >> $O/traffic.log && \
python3 scripts/pmc_summary.py $(csvdir $O/sq) > $O/sq_summary.txt && \
timeout -k 10 600 python3 bench.py --traffic-json $O/pmc_traffic.json > $O/bench.json 2> $O/bench.err
rc=$?; echo RC=$rc; cat $O/traffic.log; head -5 $(find $O/kt -name "*kernel_stats.csv") | cut -c1-200; head -4 $(find $O/kt_ref -name "*kernel_stats.csv") | cut -c1-200; head -6 $(find $O/kt_s8 -name "*kernel_stats.csv") | cut -c1-200; cut -c1-1500 $O/bench.json; exit $rc
