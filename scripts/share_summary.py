"""Summary of scripts/gpu_r06_shares.sh: per-rank GCUPS of every measured
--shard-of N share under both scorings, the slowest rank's fraction of N = 1
(C2 on the same box, mean of the runs before and after the shares) and the
N-GPU speed-up it projects (N x min share / C2: SCALE's value is the max
over ranks of the step time).
usage: share_summary.py DIR"""
import glob
import json
import os
import re
import sys


def line(path):
    with open(path) as f:
        return json.loads([l for l in f.read().splitlines() if l.strip()][-1])


def main(d):
    c2 = [line(p) for p in sorted(glob.glob(os.path.join(d, "c2_*.json")))]
    base = {"affine": sum(x["value"] for x in c2) / len(c2),
            "reference": sum(x["reference_scoring"]["value"] for x in c2) / len(c2)}
    out = {"c2_runs": {"affine": [x["value"] for x in c2],
                       "reference": [x["reference_scoring"]["value"] for x in c2]},
           "c2_mean": {k: round(v, 1) for k, v in base.items()}, "shares": {}}
    byn = {}
    for p in glob.glob(os.path.join(d, "s*_r*.json")):
        m = re.match(r"s(\d+)_r(\d+)\.json", os.path.basename(p))
        if m:
            byn.setdefault(int(m.group(1)), {})[int(m.group(2))] = line(p)
    for n, ranks in sorted(byn.items()):
        rows = {}
        for k, x in sorted(ranks.items()):
            r = x.get("reference_scoring", {})
            rows[k] = {"affine": x["value"], "reference": r.get("value"),
                       "ms_affine": x["ms_per_step"], "ms_reference": r.get("ms_per_step"),
                       "subjects": x["config"]["subjects_rank0"], "residues": x["config"]["residues_rank0"],
                       "parity": x.get("parity_sample_ok"),
                       "reference_parity": r.get("parity_ok")}
        s = {"ranks": rows, "complete": len(rows) == n}
        for sc in ("affine", "reference"):
            vals = [v[sc] for v in rows.values() if v[sc]]
            ms = [v["ms_" + sc] for v in rows.values() if v["ms_" + sc]]
            if not vals:
                continue
            s[sc] = {"min": min(vals), "max": max(vals), "slowest_rank": min(rows, key=lambda k: rows[k][sc] or 1e30),
                     "min_over_c2": round(min(vals) / base[sc], 4),
                     "mean_over_c2": round(sum(vals) / len(vals) / base[sc], 4),
                     # SCALE's value: all cells / the slowest rank's time
                     "projected_value": round(sum(v[sc] * v["ms_" + sc] for v in rows.values()) / max(ms), 1)
                     if len(rows) == n else None}
            if s[sc]["projected_value"]:
                s[sc]["projected_speedup"] = round(s[sc]["projected_value"] / base[sc], 3)
        out["shares"][n] = s
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
