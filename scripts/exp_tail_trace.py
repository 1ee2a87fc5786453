"""Tail analysis of the C2 scan: run with a -DSW_TRACE_BLOCKS build
(SW_AMD_LIB) and SW_TRACE_FILE set; reads back the per-block timeline
(start, end, HW_ID, XCC_ID | kind) and prints how many blocks are in flight
over the launch, per-CU idle at the end, and the critical blocks."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import _swpkg  # noqa: E402

sw = _swpkg.load()
path = os.environ["SW_TRACE_FILE"]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 570000
res, offs = sw.synth.database(n, shard=0)
with open(os.path.join(REPO, "tests", "golden", "queries", "P07327.fasta")) as f:
    q = sw.encode("".join(f.read().split("\n")[1:]))
h = sw.Handle(0)
db = sw.Database(h, res, offs)
m = sw.builtin_matrix(sw.MATRIX_BLOSUM62)
for _ in range(4):
    db.scan(q, matrix=m, gap_open=12, gap_extend=1)
st = db.stats()
db.close()
t = np.fromfile(path, dtype=np.uint64).reshape(-1, 4)
t0, t1 = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
ok = t1 > 0
T0 = t0[ok].min()
s, e = (t0[ok] - T0) / 100.0, (t1[ok] - T0) / 100.0  # microseconds (100 MHz)
hw, xcc, kind = t[ok, 2], t[ok, 3] & 0xffffffff, t[ok, 3] >> 32
span = e.max()
cu = (xcc << 16) | (((hw >> 13) & 7) << 8) | ((hw >> 8) & 15)  # xcc, se, cu
simd = (cu << 4) | ((hw >> 4) & 3)
out = {"blocks": int(ok.sum()), "pair_blocks": int((kind == 1).sum()), "span_us": float(span)}
# blocks in flight over time
grid = np.linspace(0, span, 41)
inflight = [int(((s <= x) & (e > x)).sum()) for x in grid]
out["inflight_every_2.5pct"] = inflight
# each SIMD's last end: how long before the kernel's end it went idle
last = {}
for k, v in zip(simd, e):
    last[k] = max(last.get(k, 0.0), v)
lv = np.array(sorted(last.values()))
out["simds_seen"] = len(lv)
out["simd_idle_tail_us_pctl"] = {p: float(span - np.percentile(lv, p)) for p in (0, 10, 50, 90, 100)}
# utilisation: sum of block durations / (simd slots x span)
out["block_us_sum"] = float((e - s).sum())
out["widest_blocks"] = [[float(a), float(b), int(k)] for a, b, k in
                        sorted(zip(s, e, kind), key=lambda x: -(x[1] - x[0]))[:8]]
out["last_blocks_end_us"] = sorted(float(x) for x in e)[-8:]
out["first_starts_us"] = sorted(float(x) for x in s)[:4] + sorted(float(x) for x in s)[2040:2052:4]
print(json.dumps(out))
