# Round 3: SQ counters of the C2 scan for each library in $LIBS (dirs under
# the package), one --pmc pass each, summarised per kernel.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r03sq}
mkdir -p $O
P=ece1782-smith-waterman-cuda_amd
B="bench.py --no-cpu-baseline --no-verify --no-reference-scoring --steps 3 --warmup 1 ${BENCH_ARGS:-}"
for lib in ${LIBS:-lib}; do
  SW_AMD_LIB=$P/$lib/libswamd.so timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $O/sq_$lib -o run --output-format csv -- python3 $B > $O/sq_$lib.json 2> $O/sq_$lib.err || { echo "sq $lib FAILED"; tail $O/sq_$lib.err; exit 1; }
  echo "== $lib"; python3 scripts/pmc_summary.py $(dirname $(find $O/sq_$lib -name run_counter_collection.csv)) | tee $O/sq_$lib.txt
done
