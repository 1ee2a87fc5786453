"""VALU instructions per wave-step (and per 128 cells) of an intra launch
from one rocprofv3 --pmc SQ pass: the dispatches whose kernel name starts
with NAME, averaged; a wave-step of sw_intra_x2<RI> is 64 lanes x RI rows x
2 subjects = 128 RI cells.  Cells per launch from a bench line of the same
workload (its cells_per_step).
usage: sq_per_step.py CSV_DIR NAME RI BENCH_JSON"""
import collections
import csv
import json
import sys


def main(d, name, ri, bench):
    ri = int(ri)
    per = collections.defaultdict(dict)
    kname = {}
    with open(d + "/run_counter_collection.csv") as f:
        for row in csv.DictReader(f):
            k = row["Kernel_Name"]
            if not k.replace("void swk::", "").startswith(name):
                continue
            disp = row["Dispatch_Id"]
            per[disp][row["Counter_Name"]] = float(row["Counter_Value"])
            per[disp]["ns"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
            kname[disp] = k.split("(")[0]
    with open(bench) as f:
        b = json.loads([l for l in f.read().splitlines() if l.strip()][-1])
    cells = b["config"]["cells_per_step"]
    rows = list(per.values())
    avg = {c: sum(r.get(c, 0) for r in rows) / len(rows) for c in rows[0]}
    valu = avg["SQ_INSTS_VALU"]
    out = {"kernel": sorted(set(kname.values())), "dispatches": len(rows), "cells_per_launch": cells,
           "sq_insts_valu_per_launch": valu, "valu_insts_per_128_cells": round(valu / (cells / 128), 4),
           "valu_insts_per_wave_step": round(valu / (cells / 128) * ri, 2),
           "profiled_ms_per_launch": round(avg["ns"] * 1e-6, 4)}
    if "GRBM_GUI_ACTIVE" in avg:
        cyc = avg["GRBM_GUI_ACTIVE"] / 8
        out["clock_ghz_under_load"] = round(cyc / avg["ns"], 3)
        out["valu_issue_frac_4.25cyc"] = round(valu * 4.25 / (1024 * cyc), 4)
    if avg.get("SQ_ACTIVE_INST_LDS"):
        out["lds_bank_conflict_cycles_per_lds_inst"] = round(avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_ACTIVE_INST_LDS"], 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
