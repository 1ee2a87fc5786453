# Parity (incl. device top-K), then SQ/LDS counters on the x2 affine kernel.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc3; mkdir -p $O
run() { name=$1; shift; SW_TUNE_SCORING=1:12:1 timeout -k 10 300 rocprofv3 --pmc "$@" -d $O/$name -o run --output-format csv -- python3 scripts/tune_inter.py x32x8 2048 > $O/$name.log 2>&1; }
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/parity.log 2>&1 && \
run a SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS && \
run b SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_LDS SQ_BUSY_CU_CYCLES && \
run c SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LEVEL_WAVES SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS && \
python3 scripts/pmc_summary.py $(for x in a b c; do dirname $(find $O/$x -name run_counter_collection.csv); done) > $O/summary.txt
rc=$?; echo RC=$rc; tail -2 $O/parity.log; cat $O/summary.txt; exit $rc
