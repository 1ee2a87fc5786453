# PMC passes over a short bench (separate rocprofv3 runs per counter group;
# no sys/runtime trace mixed with --pmc).
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
run() { name=$1; shift; timeout -k 10 300 rocprofv3 --pmc "$@" -d gpurun_out/pmc/$name -o run --output-format csv -- $B > gpurun_out/pmc/$name.log 2>&1; }
run p1 FETCH_SIZE && \
run p2 WRITE_SIZE && \
run p3 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE && \
run p4 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU && \
run p5 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM && \
run p6 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
echo "RC=$?"
