"""Per-query timeline of a C3 batch from a rocprofv3 kernel trace: each
query's fp16 inter launch, the kernels after it until the next query's
fp16 launch (the rescue tail) and the idle gaps.
usage: c3_timeline.py KERNEL_TRACE.csv"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
t0 = ks[0][0]
short = lambda n: n.split("(")[0].replace("void ", "").replace("swk::", "")[:60]
tot = collections.defaultdict(float)
for s, e, n in ks:
    tot[short(n)] += (e - s) / 1e6
for n, v in sorted(tot.items(), key=lambda x: -x[1])[:15]:
    print("%10.2f ms  %s" % (v, n))
# the main scan launches: sw_inter_x2p (merged) with f16
main = [(s, e, n) for s, e, n in ks if "sw_inter_x2p" in n and "true, true, true" in n.replace("ELb1", "true")]
print("main launches:", len(main))
for i, (s, e, n) in enumerate(main):
    nxt = main[i + 1][0] if i + 1 < len(main) else ks[-1][1]
    after = [(a, b, m) for a, b, m in ks if a >= e and a < nxt]
    busy_end = max([b for a, b, m in ks if a < nxt] + [e])
    print("%3d start %8.2f ms dur %6.2f ms, next main +%6.2f ms after end; %d kernels between: %s" % (
        i, (s - t0) / 1e6, (e - s) / 1e6, (nxt - e) / 1e6, len(after),
        ", ".join("%s %.2f" % (short(m)[:28], (b - a) / 1e6) for a, b, m in after[:6])))
