set -o pipefail
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
run() { name=$1; var=$2; shift 2; SW_INTER_VARIANT=$var timeout -k 10 300 rocprofv3 --pmc "$@" -d gpurun_out/pmc2/$name -o run --output-format csv -- python3 scripts/tune_inter.py $var 1536 > gpurun_out/pmc2/$name.log 2>&1; }
for v in 64x8 p64x8; do
run a_$v $v SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU_INT32 SQ_WAVE_CYCLES && \
run b_$v $v SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_LDS SQ_BUSY_CU_CYCLES && \
run c_$v $v SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LEVEL_WAVES SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD || exit 1
done
echo RC=0
