"""Block timeline of one rank's share of a strong-scaled C2 database (run
with a -DSW_TRACE_BLOCKS build via SW_AMD_LIB and SW_TRACE_FILE set):
blocks in flight over the launch, block durations against their width and
form (single wave / group), the critical blocks.
usage: exp_share_trace.py SHARD_OF [LONG_THRESHOLD] [ref]
(ref: the reference's scoring, BLOSUM50 linear 2, instead of BLOSUM62 11/1)"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import _swpkg  # noqa: E402

sw = _swpkg.load()
path = os.environ["SW_TRACE_FILE"]
S = int(sys.argv[1]) if len(sys.argv) > 1 else 8
T = int(sys.argv[2]) if len(sys.argv) > 2 else 0
res, offs = sw.synth.database(570000, shard=0)
_, r, o = sw.dist.shard(res, offs, 0, S)
with open(os.path.join(REPO, "tests", "golden", "queries", "P07327.fasta")) as f:
    q = sw.encode("".join(f.read().split("\n")[1:]))
h = sw.Handle(0)
db = sw.Database(h, r, o, long_threshold=(T or None))
REF = len(sys.argv) > 3 and sys.argv[3] == "ref"
m = sw.builtin_matrix(sw.MATRIX_BLOSUM50_REF if REF else sw.MATRIX_BLOSUM62)
go, ge = (2, 2) if REF else (12, 1)
for _ in range(4):
    db.scan(q, matrix=m, gap_open=go, gap_extend=ge)
st = db.stats()
tm = h.timing()
db.close()
t = np.fromfile(path, dtype=np.uint64).reshape(-1, 4)
tall = t
t = t[:st["n_blocks"]]
t0, t1 = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
ok = t1 > 0
T0 = t0[ok].min()
s, e = (t0[ok] - T0) / 100.0, (t1[ok] - T0) / 100.0  # microseconds (100 MHz)
kind = t[ok, 3] >> 32
blk = np.nonzero(ok)[0]
lens = np.sort(o[1:] - o[:-1])[::-1][st["n_long"]:]
width = np.array([lens[b * 64] for b in blk])  # longest subject of the block
span = e.max()
out = {"shard_of": S, "long_threshold": st["long_threshold"], "n_long": st["n_long"], "blocks": int(ok.sum()),
       "group_blocks": int((kind == 1).sum()), "span_us": round(float(span), 1), "timing_ms": tm}
grid = np.linspace(0, span, 21)
out["inflight_every_5pct"] = [int(((s <= x) & (e > x)).sum()) for x in grid]
dur = e - s
for kd in (0, 1):
    sel = kind == kd
    if sel.any():
        ww = width[sel]
        out["form%d" % kd] = {"n": int(sel.sum()), "width_min_max": [int(ww.min()), int(ww.max())],
                              "dur_us_min_med_max": [round(float(np.min(dur[sel])), 1),
                                                     round(float(np.median(dur[sel])), 1),
                                                     round(float(np.max(dur[sel])), 1)],
                              "us_per_column_med": round(float(np.median(dur[sel] / ww)), 3),
                              "start_us_max": round(float(s[sel].max()), 1)}
crit = np.argsort(-e)[:6]
out["last_to_end"] = [[int(blk[i]), int(kind[i]), int(width[i]), round(float(s[i]), 1), round(float(e[i]), 1)]
                      for i in crit]
print(json.dumps(out))

# merged launch (sw_scan_lpt): per-workgroup records after the per-block ones
nb = st["n_blocks"]
w = tall[nb:]
okw = w[:, 1] > 0
if okw.any():
    ws = (w[okw, 0].astype(np.int64) - T0) / 100.0
    we = (w[okw, 1].astype(np.int64) - T0) / 100.0
    wk = w[okw, 3] >> 32
    lpt = {"workgroups": int(okw.sum())}
    for kd, name in ((2, "inter"), (3, "intra")):
        sel = wk == kd
        if sel.any():
            d = we[sel] - ws[sel]
            lpt[name] = {"n": int(sel.sum()), "start_us_max": round(float(ws[sel].max()), 1),
                         "end_us_max": round(float(we[sel].max()), 1),
                         "dur_us_min_med_max": [round(float(d.min()), 1), round(float(np.median(d)), 1),
                                                round(float(d.max()), 1)]}
    grid = np.linspace(0, float(we.max()), 21)
    lpt["wgs_inflight_every_5pct"] = [int(((ws <= x) & (we > x)).sum()) for x in grid]
    last = np.argsort(-we)[:6]
    lpt["last_to_end"] = [[int(wk[i]), round(float(ws[i]), 1), round(float(we[i]), 1)] for i in last]
    print(json.dumps({"lpt": lpt}))
