# Round 2: SQ counters of the merged launch on the C2/8 share vs the full C2
# per-wave kernel (VALU per cell, VALU issue utilisation, stall split).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02v}
mkdir -p $O
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
B="bench.py --no-cpu-baseline --no-verify --no-reference-scoring --steps 3 --warmup 1"
timeout -s KILL 200 rocprofv3 --pmc $C -d $O/s8 -o run --output-format csv -- python3 $B --shard-of 8 > $O/s8.json 2> $O/s8.err && \
timeout -s KILL 200 rocprofv3 --pmc $C -d $O/c2 -o run --output-format csv -- python3 $B > $O/c2.json 2> $O/c2.err
rc=$?; echo RC=$rc
for d in s8 c2; do f=$(find $O/$d -name run_counter_collection.csv); echo "== $d"; python3 - "$f" <<'PY'
import csv,sys,collections
s=collections.defaultdict(float); n=collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k=r['Kernel_Name']
    if 'sw_' not in k: continue
    s[(k[:44],r['Counter_Name'])]+=float(r['Counter_Value']); n[(k[:44],r['Counter_Name'])]+=1
for (k,c),v in sorted(s.items()): print(k,c,'%.4g'%(v/max(1,n[(k,c)])))
PY
done; exit $rc
