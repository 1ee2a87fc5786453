# Round 6 A/B: the pair-image intra form (sw_intra_x2w,
# (S, 1) dwords, 8 waves sharing 133 KB at RI 20; lib_wide, built with
# IX2FLAGS=-DSW_IX2_WIDE=1) against sw_intra_x2 on C5, alternating, both
# scorings per line; the intra GPU tests on lib_wide first; then an SQ pass
# (VALU per wave-step) of each form's C5 launch.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06c5wide}
mkdir -p $O
LW=$PWD/ece1782-smith-waterman-cuda_amd/lib_wide/libswamd.so
SW_AMD_LIB=$LW timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "intra" --timeout 200 --timeout-method thread > $O/wide_tests.log 2>&1 || { echo WIDE TESTS FAILED; tail -30 $O/wide_tests.log; exit 1; }
tail -1 $O/wide_tests.log
B="bench.py --config c5 --no-cpu-baseline --sustained-seconds 0"
run() { tag=$1; lib=$2; SW_AMD_LIB=$lib timeout -k 10 300 python3 $B > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -10 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$tag', d['value'], d['ms_per_step'], r.get('value'), d.get('parity_sample_ok'), r.get('parity_ok'), d['kernels'])"; }
LD=$PWD/ece1782-smith-waterman-cuda_amd/lib/libswamd.so
run c5_base1 $LD && run c5_wide1 $LW && run c5_base2 $LD && run c5_wide2 $LW || exit 1
P="bench.py --config c5 --no-cpu-baseline --no-verify --no-reference-scoring --sustained-seconds 0 --steps 3 --warmup 1"
SQ="SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
SW_AMD_LIB=$LW timeout -s KILL 200 rocprofv3 --pmc $SQ -d $O/sq_wide -o run --output-format csv -- python3 $P > $O/sq_wide.json 2> $O/sq_wide.err || { echo SQ WIDE FAILED; tail -5 $O/sq_wide.err; exit 1; }
SW_AMD_LIB=$LD timeout -s KILL 200 rocprofv3 --pmc $SQ -d $O/sq_base -o run --output-format csv -- python3 $P > $O/sq_base.json 2> $O/sq_base.err || { echo SQ BASE FAILED; tail -5 $O/sq_base.err; exit 1; }
for f in wide base; do python3 scripts/sq_per_step.py $(dirname $(find $O/sq_$f -name run_counter_collection.csv)) sw_intra_x2 20 $O/c5_base1.json > $O/sq_$f.txt; echo $f; cat $O/sq_$f.txt; done
echo RC=0
