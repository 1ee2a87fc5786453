"""The merged launch's pipelined long pair measured alone: two subjects of
LEN residues (plus one block of 64 200-residue ones: the merged launch needs a wave-pair block) against P07327, in one
sw_scan_lpt launch, so the scan time is the pair's latency with the GPU
otherwise idle.  Compare with the pair's span inside the 1/8 share's launch
(scripts/exp_share_dump.py) to see how much the co-resident waves slow it.
usage: exp_pipe_alone.py [LEN] [ref]   (SW_LPT_PIPE=0 / 1 picks the form)"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import _swpkg  # noqa: E402

sw = _swpkg.load()
L = int(sys.argv[1]) if len(sys.argv) > 1 else 7429
REF = len(sys.argv) > 2 and sys.argv[2] == "ref"
rng = np.random.default_rng(1)
lens = np.array([L, L - 40] + [200] * 64, dtype=np.int64)
offs = np.zeros(len(lens) + 1, dtype=np.int64)
offs[1:] = np.cumsum(lens)
res = rng.integers(0, 20, size=int(offs[-1]), dtype=np.uint8)
with open(os.path.join(REPO, "tests", "golden", "queries", "P07327.fasta")) as f:
    q = sw.encode("".join(f.read().split("\n")[1:]))
h = sw.Handle(0)
db = sw.Database(h, res, offs, long_threshold=1024)
m = sw.builtin_matrix(sw.MATRIX_BLOSUM50_REF if REF else sw.MATRIX_BLOSUM62)
go, ge = (2, 2) if REF else (12, 1)
for _ in range(3):
    db.scan(q, matrix=m, gap_open=go, gap_extend=ge)
h.timing_reset()
for _ in range(20):
    db.scan(q, matrix=m, gap_open=go, gap_extend=ge)
t = h.timing_total()
us = t["total_ms"] / t["scans"] * 1e3
print(json.dumps({"len": L, "ref": REF, "kernel": h.last_kernel(), "scan_us": round(us, 1),
                  "ns_per_step": round(us * 1e3 / (L + 63), 2), "pipe": os.environ.get("SW_LPT_PIPE")}))
db.close()
