"""CU-level idleness of a merged launch from an exp_share_dump.py trace
(.npz): with two 4-wave workgroups per CU every SIMD holds two waves, and a
VALU-bound wave alone on its SIMD issues nearly as fast as two together, so
the time a CU holds ZERO workgroups is the launch's real loss, while one
workgroup (one wave per SIMD) mostly is not (the trace's single-wave items
run ~2.2x faster then: scripts/lpt_fit.py's bimodal ratios).  Prints the
share of CU-time with 0 and 1 workgroups, overall and in the last 10 %.
usage: trace_cu_idle.py TRACE.npz"""
import json
import sys

import numpy as np

z = np.load(sys.argv[1])
t = z["trace"]
nb = int(z["n_blocks"])
b, w = t[:nb], t[nb:]
w = w[w[:, 1] > 0]
T0 = b[b[:, 1] > 0, 0].astype(np.int64).min()
ws = (w[:, 0].astype(np.int64) - T0) / 100.0
we = (w[:, 1].astype(np.int64) - T0) / 100.0
hw = w[:, 2].astype(np.int64)
cu = (w[:, 3] & 0xffffffff).astype(np.int64) * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 8) & 0xf)
span = float(we.max())
ucu = np.unique(cu)
tot = {0: 0.0, 1: 0.0}
last = {0: 0.0, 1: 0.0}
t10 = 0.9 * span
for c in ucu:
    m = cu == c
    ev = sorted([(float(s), 1) for s in ws[m]] + [(float(e), -1) for e in we[m]])
    n, prev = 0, 0.0
    for x, d in ev + [(span, 0)]:
        x = max(x, 0.0)
        if n in tot and x > prev:
            tot[n] += x - prev
            lo = max(prev, t10)
            if x > lo:
                last[n] += x - lo
        n += d
        prev = max(prev, x)
denom = len(ucu) * span
print(json.dumps({"cus": int(len(ucu)), "span_us": round(span, 1),
                  "cu_time_pct_with_0_wg": round(100 * tot[0] / denom, 2),
                  "cu_time_pct_with_1_wg": round(100 * tot[1] / denom, 2),
                  "last10_cu_time_pct_with_0_wg": round(100 * last[0] / denom, 2),
                  "last10_cu_time_pct_with_1_wg": round(100 * last[1] / denom, 2)}))
