#!/usr/bin/env python3
"""Sweep inter-kernel shapes (SW_INTER_VARIANT) and long thresholds on the
C2 workload in one process; every result must equal the first one."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import _swpkg  # noqa: E402

sw = _swpkg.load()
variants = (sys.argv[1] if len(sys.argv) > 1 else "32x8,32x16,16x16,48x8,64x8").split(",")
thresholds = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "3072,2048,1536,1024").split(",")]
qname = sys.argv[3] if len(sys.argv) > 3 else "P07327"
nseq = int(sys.argv[4]) if len(sys.argv) > 4 else 570000
reps = 5
# scoring: SW_TUNE_SCORING="<matrix id>:<gap open>:<gap extend>" (default the
# reference's BLOSUM50, linear gap 2)
mid, go, ge = (int(x) for x in os.environ.get("SW_TUNE_SCORING", "0:2:2").split(":"))
mat = sw.capi.builtin_matrix(mid)
res, offs = sw.synth.database(nseq, shard=0)
with open(os.path.join(REPO, "tests/golden/queries/%s.fasta" % qname)) as f:
    q = sw.encode("".join(f.read().split("\n")[1:]))
h = sw.Handle(0)
db = sw.Database(h, res, offs)
ref = None
cells = len(q) * float(offs[-1])
for thr in thresholds:
    db.set_long_threshold(thr)
    st = db.stats()
    for v in variants:
        os.environ["SW_INTER_VARIANT"] = v
        out = db.scan(q, mat, go, ge)  # warm
        if ref is None:
            ref = out
        ok = bool(np.array_equal(out, ref))
        h.timing_reset()
        t = time.perf_counter()
        for _ in range(reps):
            db.scan(q, mat, go, ge)
        wall = (time.perf_counter() - t) / reps
        kt = h.timing_total()
        n = kt["scans"]
        rec = {"scoring": [mid, go, ge], "variant": v, "long_threshold": thr, "n_long": st["n_long"], "ok": ok,
               "inter_ms": round(kt["inter_ms"] / n, 3), "intra_ms": round(kt["intra_ms"] / n, 3),
               "scan_ms": round(kt["total_ms"] / n, 3), "wall_ms": round(wall * 1e3, 3),
               "gcups_scan": round(cells / (kt["total_ms"] / n * 1e-3) / 1e9, 1)}
        print(json.dumps(rec), flush=True)
