#!/usr/bin/env python3
"""Per-step timeline of a rocprofv3 --kernel-trace (run_kernel_trace.csv):
groups the dispatches into steps at each occurrence of the step's first
kernel (default: the scan launch) and prints, per kernel position in the
step, its average duration and the average idle gap before it on its queue,
plus the average step period.  usage: step_gaps.py TRACE.csv [FIRST_KERNEL_SUBSTR]"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "sw_build_profile"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", r.get("Stream_Id", "?"))))
    rows.sort()
    steps, cur = [], None
    for r in rows:
        if first in r[2]:
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append(r)
    steps = steps[2:-1]  # drop warm-up edges and the unfinished last
    dur, gap, cnt = defaultdict(float), defaultdict(float), defaultdict(int)
    periods = []
    for i, st in enumerate(steps):
        if i + 1 < len(steps):
            periods.append(steps[i + 1][0][0] - st[0][0])
        last_end = {}
        for k, (s, e, name, q) in enumerate(st):
            key = "%02d %s [q%s]" % (k, name.split("(")[0][:70], q)
            dur[key] += e - s
            if q in last_end:
                gap[key] += s - last_end[q]
            cnt[key] += 1
            last_end[q] = e
    n = max(len(steps), 1)
    print("steps %d, period %.1f us" % (len(steps), sum(periods) / max(len(periods), 1) / 1e3))
    for key in sorted(dur):
        print("%-90s dur %8.1f us  gap-before %7.1f us  (%d)" % (key, dur[key] / cnt[key] / 1e3, gap[key] / cnt[key] / 1e3, cnt[key]))


if __name__ == "__main__":
    main()
