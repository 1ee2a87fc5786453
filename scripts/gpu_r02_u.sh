# Round 2: SQ counters of the C5 intra kernel (what bounds it: VALU issue,
# issue stalls or waits), affine and reference scoring.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02u}
mkdir -p $O
B="bench.py --no-cpu-baseline --no-verify --config c5 --steps 3 --warmup 1"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/sq1 -o run --output-format csv -- python3 $B --no-reference-scoring > $O/sq1.json 2> $O/sq1.err && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -d $O/sq2 -o run --output-format csv -- python3 $B --no-reference-scoring > $O/sq2.json 2> $O/sq2.err
rc=$?; echo RC=$rc
for d in sq1 sq2; do f=$(find $O/$d -name run_counter_collection.csv); python3 - "$f" <<'PY'
import csv,sys,collections
s=collections.defaultdict(float); n=collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k=r['Kernel_Name']
    if 'sw_intra' not in k: continue
    s[(k[:40],r['Counter_Name'])]+=float(r['Counter_Value']); n[(k[:40],r['Counter_Name'])]+=1
for (k,c),v in sorted(s.items()): print(k,c,'%.4g'%(v/ max(1,n[(k,c)]) * 1),'(per dispatch-row avg)')
PY
done; exit $rc
