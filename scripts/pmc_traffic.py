#!/usr/bin/env python3
"""Per-launch HBM bytes of the bench's dominant kernel from two rocprofv3
--pmc passes (FETCH_SIZE and WRITE_SIZE cannot share one pass on gfx950).

FETCH_SIZE / WRITE_SIZE are reported in KiB.  Per MI355X_MICROARCH.md (HBM
section), on gfx950 FETCH_SIZE counts half the bytes of a wide (16 B/lane)
streaming read, which is how sw_inter loads its packed residue groups, so it
is doubled; WRITE_SIZE is taken as reported.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR WORKLOAD_KEY OUT_JSON ROCPROF_NAME_SUBSTR LABEL [SQ_DIR|-] [NSCANS]
(LABEL = the library's kernel name, sw_last_kernel(), which bench.py matches;
SQ_DIR: a pass with SQ_INSTS_VALU and GRBM_GUI_ACTIVE for the VALU issue
fraction of the same kernel, and SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS
when the pass has them)
OUT_JSON is merged, not overwritten: every workload's entry lands under
"workloads"[WORKLOAD_KEY] (bench.py looks its own key up there); the headline
C2 entry (a key without a "cN:" config prefix) is also the file's top level.
"""
import csv
import datetime
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def per_dispatch(d, counter, kernel):
    vals = []
    with open(d + "/run_counter_collection.csv") as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit("no %s rows for %s in %s" % (counter, kernel, d))
    return vals


def durations(d, kernel):
    out = []
    with open(d + "/run_counter_collection.csv") as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == "SQ_INSTS_VALU":
                out.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return out


def main():
    fdir, wdir, key, out, kernel, label = sys.argv[1:7]
    sqdir = sys.argv[7] if len(sys.argv) > 7 and sys.argv[7] != "-" else None
    # scans profiled per pass (0: one dispatch of the kernel per scan): a
    # batch's queries dispatch different kernels of one family, so their
    # counters are summed and divided by the scans
    nscans = int(sys.argv[8]) if len(sys.argv) > 8 else 0
    f = per_dispatch(fdir, "FETCH_SIZE", kernel)
    w = per_dispatch(wdir, "WRITE_SIZE", kernel)

    def mean(v):
        return sum(v) / (nscans or len(v))
    fetch = mean(f) * 1024 * 2
    write = mean(w) * 1024
    res = {"workload_key": key, "kernel": label, "rocprof_kernel": kernel,
           "fetch_bytes_per_launch": round(fetch), "write_bytes_per_launch": round(write),
           "hbm_bytes_per_launch": round(fetch + write),
           "dispatches": {"fetch_pass": len(f), "write_pass": len(w)},
           "per": "scan (%d scans per pass, every dispatch of the kernel family summed)" % nscans if nscans
                  else "launch",
           "raw_kib_mean": {"FETCH_SIZE": mean(f), "WRITE_SIZE": mean(w)},
           "correction": "FETCH_SIZE x2 (gfx950, 16 B/lane streaming reads); WRITE_SIZE as reported",
           # bench.py reports the bytes only for a build with these kernel sources
           "kernel_src_sha16": __import__("bench").kernel_source_hash(),
           "measured": datetime.date.today().isoformat()}
    if sqdir:
        v = per_dispatch(sqdir, "SQ_INSTS_VALU", kernel)
        g = per_dispatch(sqdir, "GRBM_GUI_ACTIVE", kernel)
        dn = durations(sqdir, kernel)
        res["sq_insts_valu_per_launch"] = round(mean(v))
        # GRBM_GUI_ACTIVE counts the GPU's cycles during each dispatch: per
        # scan it sums like the durations
        res["grbm_gui_active_per_launch"] = round(mean(g))
        res["profiled_ns_per_launch"] = round(sum(dn) / (nscans or len(dn))) if dn else None
        for c in ("SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS"):
            try:
                x = per_dispatch(sqdir, c, kernel)
                res[c.lower() + "_per_launch"] = round(mean(x))
            except SystemExit:
                pass
    try:
        with open(out) as fi:
            doc = json.load(fi)
    except (OSError, ValueError):
        doc = {}
    works = dict(doc.get("workloads", {}))
    if doc.get("workload_key") and doc["workload_key"] not in works:
        works[doc["workload_key"]] = {k: v for k, v in doc.items() if k != "workloads"}
    works[key] = res
    top = res if ":" not in key.split("/")[0] else {k: v for k, v in doc.items() if k != "workloads"}
    top = dict(top)
    top["workloads"] = works
    with open(out, "w") as fo:
        json.dump(top, fo, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
