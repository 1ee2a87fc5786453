# Round 6: SQ counters of C2's merged launch under the reference scoring
# (BLOSUM50, linear gap 2): VALU and LDS issue, LDS instructions and bank
# conflicts, with a kernel trace of the same command.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06sqref}
mkdir -p $O
B="bench.py --matrix blosum50 --gap-open 2 --gap-extend 2 --no-reference-scoring --no-verify --no-cpu-baseline --sustained-seconds 0 --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $B > $O/kt.json 2> $O/kt.err || { echo TRACE FAILED; tail -5 $O/kt.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $O/sq -o run --output-format csv -- python3 $B > $O/sq.json 2> $O/sq.err || { echo SQ FAILED; tail -5 $O/sq.err; exit 1; }
python3 scripts/pmc_summary.py $(dirname $(find $O/sq -name run_counter_collection.csv)) > $O/sq_summary.txt
cat $O/sq_summary.txt
cp $(find $O/kt -name "*kernel_stats.csv") $O/kernel_stats.csv
head -4 $O/kernel_stats.csv | cut -c1-160
echo RC=0
