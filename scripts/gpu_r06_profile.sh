# Round 6 profiles of the bench configs in $CFGS (default "c2 c5 c3"): per
# config a kernel trace with stats, two PMC passes (FETCH_SIZE, WRITE_SIZE)
# and one SQ pass (VALU instructions, LDS bank conflicts, wave cycles) of its
# dominant kernel, merged into $O/pmc_traffic.json (scripts/pmc_traffic.py),
# then the bench line of each config reading it.  The dominant kernel's
# rocprof name is the top of the trace's kernel stats; its library label is
# the bench line's roofline kernel.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06prof}
mkdir -p $O
cp pmc_traffic.json $O/pmc_traffic.json
B="bench.py --no-cpu-baseline --no-verify --no-reference-scoring --sustained-seconds 0"
csvdir() { dirname $(find $1 -name run_counter_collection.csv); }
for c in ${CFGS:-c2 c5 c3}; do
  # NS: scans per profiled run when the dominant work is a family of kernels (C3: 20 queries x 5 steps: the cold first step, 1 warm-up, 1 timed, the two cold/warm steps)
  case $c in c2) a="" ; s="--steps 3 --warmup 1" ; NS=0 ;; c5) a="--config c5" ; s="--steps 3 --warmup 1" ; NS=0 ;; c3) a="--config c3" ; s="--steps 1 --warmup 1" ; NS=100 ;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$c -o run --output-format csv -- python3 $B $a $s > $O/kt_$c.json 2> $O/kt_$c.err || { echo "TRACE $c FAILED"; tail -5 $O/kt_$c.err; exit 1; }
  KN=$(python3 -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
print(rows[0]['Name'].split('(')[0].replace('void swk::',''))" $(find $O/kt_$c -name "*kernel_stats.csv"))
  LABEL=$(python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1])
print(d['roofline']['kernel'])" $O/kt_$c.json)
  KEY=$(python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1])
print(d['roofline']['workload_key'])" $O/kt_$c.json)
  # (a batch: every scan's dominant kernel summed, the merged launches when
  # the batch's label says so, else the inter kernels)
  [ $NS -gt 0 ] && { case "$LABEL" in *+lpt*) KN="sw_scan_lpt" ;; *) KN="sw_inter_x2" ;; esac; }
  echo "$c: rocprof '$KN' label '$LABEL' key '$KEY'"
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$c -o run --output-format csv -- python3 $B $a $s > $O/fetch_$c.json 2> $O/fetch_$c.err && \
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/write_$c -o run --output-format csv -- python3 $B $a $s > $O/write_$c.json 2> $O/write_$c.err && \
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $O/sq_$c -o run --output-format csv -- python3 $B $a $s > $O/sq_$c.json 2> $O/sq_$c.err && \
  python3 scripts/pmc_traffic.py $(csvdir $O/fetch_$c) $(csvdir $O/write_$c) "$KEY" $O/pmc_traffic.json "$KN" "$LABEL" $(csvdir $O/sq_$c) $NS >> $O/traffic.log && \
  python3 scripts/pmc_summary.py $(csvdir $O/sq_$c) > $O/sq_summary_$c.txt || { echo "PMC $c FAILED"; tail -5 $O/*_$c.err; exit 1; }
done
for c in ${CFGS:-c2 c5 c3}; do
  case $c in c2) a="" ;; c5) a="--config c5" ;; c3) a="--config c3" ;; esac
  timeout -k 10 600 python3 bench.py $a --no-cpu-baseline --traffic-json $O/pmc_traffic.json > $O/bench_$c.json 2> $O/bench_$c.err || { echo "BENCH $c FAILED"; tail -5 $O/bench_$c.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); r=d['roofline']
print(sys.argv[2], d['value'], r['kernel'], r.get('traffic'), r.get('frac'), json.dumps(d.get('valu_hw')))" $O/bench_$c.json $c
done
echo RC=0
