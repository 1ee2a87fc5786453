#!/usr/bin/env python3
"""Per-workgroup timeline of one merged longest-first launch (sw_scan_lpt)
from an exp_share_dump.py npz: in-flight curve, the workgroups that end
last (their LPT rank = grid index, kind, start, duration), and per kind the
duration against the rank.  usage: exp_lpt_trace.py TRACE.npz"""
import json
import sys

import numpy as np

z = np.load(sys.argv[1])
t = z["trace"]
nb = int(z["n_blocks"])
w = t[nb:]
ok = w[:, 1] > 0
idx = np.nonzero(ok)[0]
s = w[ok, 0].astype(np.int64)
e = w[ok, 1].astype(np.int64)
T0 = s.min()
s = (s - T0) / 100.0
e = (e - T0) / 100.0
kind = (w[ok, 3] >> 32).astype(int)
d = e - s
span = e.max()
print("workgroups %d (inter %d, intra %d), span %.1f us" % (len(s), (kind == 2).sum(), (kind == 3).sum(), span))
grid = np.linspace(0, span, 21)
print("in flight every 5%%:", [int(((s <= x) & (e > x)).sum()) for x in grid])
work = d.sum()
print("sum of durations %.0f us = %.1f us over 512 slots (span %.1f): slot utilisation %.1f%%"
      % (work, work / 512, span, 100 * work / 512 / span))
last = np.argsort(-e)[:16]
print("last to end: rank kind start dur end")
for i in last:
    print("  %4d %s %7.1f %7.1f %7.1f" % (idx[i], "inter" if kind[i] == 2 else "intra", s[i], d[i], e[i]))
for k, name in ((2, "inter"), (3, "intra")):
    sel = kind == k
    r = idx[sel]
    print(name, "rank<32 dur:", np.round(d[sel][np.argsort(r)][:32], 0).astype(int).tolist())
    print(name, "start of rank>=400 (min):", round(float(s[sel][r >= 400].min()), 1) if (r >= 400).any() else None)
