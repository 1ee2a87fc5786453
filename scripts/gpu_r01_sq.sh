# SQ counters of the final kernels: C2 (merged scan + intra) and C5 (intra).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sq; mkdir -p $O
run() { name=$1; cfg=$2; shift 2; timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/$name -o run --output-format csv -- python3 bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-reference-scoring > $O/$name.log 2>&1; }
run c2a c2 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS && \
run c2b c2 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES && \
run c5a c5 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS && \
run c5b c5 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES && \
python3 scripts/pmc_summary.py $(for x in c2a c2b; do dirname $(find $O/$x -name run_counter_collection.csv); done) > $O/c2_summary.txt && \
python3 scripts/pmc_summary.py $(for x in c5a c5b; do dirname $(find $O/$x -name run_counter_collection.csv); done) > $O/c5_summary.txt
rc=$?; echo RC=$rc; cat $O/c2_summary.txt | head -40; cat $O/c5_summary.txt | head -30; exit $rc
