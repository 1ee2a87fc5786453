# Round 5 A/B: C2 with the merged launch's wave groups
# widened to every block (pairs: every pass boundary inside a round goes
# through LDS, only round-to-round through HBM; quads: one HBM hand-off per
# four passes) against the default (single waves below the pair width):
# GCUPS and the dominant kernel's HBM bytes per launch (FETCH_SIZE x2 +
# WRITE_SIZE) for each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r05ab_groups}
mkdir -p $O
B="bench.py --no-cpu-baseline --no-verify --no-reference-scoring --sustained-seconds 0"
csvdir() { dirname $(find $1 -name run_counter_collection.csv); }
for v in default pairs quads; do
  case $v in default) E="" ;; pairs) E="SW_PAIR_WIDTH=16 SW_QUAD_WIDTH=0" ;; quads) E="SW_PAIR_WIDTH=16 SW_QUAD_WIDTH=16" ;; esac
  env $E timeout -k 10 300 python3 $B > $O/$v.json 2> $O/$v.err || { echo "$v FAILED"; tail -5 $O/$v.err; exit 1; }
  env $E timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$v -o run --output-format csv -- python3 $B --steps 3 --warmup 1 > /dev/null 2> $O/fetch_$v.err && \
  env $E timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/write_$v -o run --output-format csv -- python3 $B --steps 3 --warmup 1 > /dev/null 2> $O/write_$v.err || { echo "PMC $v FAILED"; exit 1; }
  python3 - $O/$v.json $(csvdir $O/fetch_$v) $(csvdir $O/write_$v) $v <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
def m(path, c):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path + "/run_counter_collection.csv"))
         if "sw_scan_lpt" in r["Kernel_Name"] and r["Counter_Name"] == c]
    return sum(v) / len(v) * 1024
f, w = m(sys.argv[2], "FETCH_SIZE") * 2, m(sys.argv[3], "WRITE_SIZE")
print(sys.argv[4], d["value"], d["ms_per_step"], d["kernels"]["inter"], "HBM GB/launch %.2f (fetch %.2f write %.2f)" % ((f + w) / 1e9, f / 1e9, w / 1e9))
PY
done
echo RC=0
