#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs per kernel (mean over dispatches).
usage: pmc_summary.py DIR [DIR...]   (each DIR holds run_counter_collection.csv)"""
import csv
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for d in sys.argv[1:]:
    with open(d + "/run_counter_collection.csv") as f:
        for row in csv.DictReader(f):
            k = row["Kernel_Name"]
            if "sw_" not in k:
                continue
            k = k.split("(")[0].replace("void swk::", "")
            agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
            dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
for k, cs in agg.items():
    print(k, " mean dispatch ns (profiled):", sum(dur[k]) / len(dur[k]))
    for c, v in sorted(cs.items()):
        print("   %-24s %.6g" % (c, sum(v) / len(v)))
