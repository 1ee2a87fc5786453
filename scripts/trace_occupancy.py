"""Workgroup-slot occupancy of a merged launch from an exp_share_dump.py
trace (.npz): idle slot-time overall and in the launch's last 10 %, the mean
occupancy between 5 and 80 % of the span, and the gap between a workgroup's
end and the next start on the same CU (HW_ID bits 8-15 and XCC_ID).
usage: trace_occupancy.py TRACE.npz [SLOTS=512]"""
import json
import sys

import numpy as np

z = np.load(sys.argv[1])
slots = int(sys.argv[2]) if len(sys.argv) > 2 else 512
t = z["trace"]
nb = int(z["n_blocks"])
b = t[:nb]
ok = b[:, 1] > 0
T0 = b[ok, 0].astype(np.int64).min()
w = t[nb:]
okw = w[:, 1] > 0
ws = (w[okw, 0].astype(np.int64) - T0) / 100.0  # us (100 MHz stamps)
we = (w[okw, 1].astype(np.int64) - T0) / 100.0
cu = ((w[okw, 2].astype(np.int64) >> 8) & 0xFF) | ((w[okw, 3].astype(np.int64) & 0xF) << 8)
span = float(we.max())
xs = np.linspace(0, span, 4000)
occ = np.array([((ws <= x) & (we > x)).sum() for x in xs])
dt = span / len(xs)
idle = (slots - occ).clip(0)
gaps = []
for c in np.unique(cu):
    m = cu == c
    s, e = ws[m], we[m]
    for x in e:
        nxt = s[s >= x - 0.01]
        if len(nxt) and x < 0.85 * span:
            gaps.append(float(nxt.min() - x))
gaps = np.array(gaps)
out = {"entries": int(okw.sum()), "span_us": round(span, 1),
       "idle_pct": round(100 * idle.sum() * dt / (slots * span), 2),
       "idle_last10_pct": round(100 * idle[xs > 0.9 * span].sum() * dt / (slots * span), 2),
       "mean_occupancy_5_80": round(float(occ[(xs > 0.05 * span) & (xs < 0.8 * span)].mean()), 1),
       "cu_gap_us_median_p90_mean": [round(float(np.median(gaps)), 1), round(float(np.percentile(gaps, 90)), 1),
                                     round(float(gaps.mean()), 1)] if len(gaps) else None}
print(json.dumps(out))
