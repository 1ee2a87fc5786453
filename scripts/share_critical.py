"""Critical path of a merged launch from an exp_share_dump.py trace (.npz):
slot-time by item kind (inter / intra workgroups), each inter form's block
widths and durations (4 = quads, 3 = tris, 1 = pairs, 0 = single waves), when the
intra items start, workgroups in flight every 5 % of the span and the last
entries to end.
usage: share_critical.py TRACE.npz"""
import json
import sys

import numpy as np


def main(path):
    z = np.load(path)
    t = z["trace"]
    nb = int(z["n_blocks"])
    b, w = t[:nb], t[nb:]
    T0 = b[b[:, 1] > 0, 0].astype(np.int64).min()
    ok = w[:, 1] > 0
    ws = (w[:, 0].astype(np.int64) - T0) / 100.0  # us (100 MHz)
    we = (w[:, 1].astype(np.int64) - T0) / 100.0
    kind = (w[:, 3] >> 32).astype(int)
    span = float(we[ok].max())
    out = {"kernel": str(z["kernel"]), "blocks": nb, "long_subjects": int(z["n_long"]),
           "long_threshold": json.loads(str(z["stats"])).get("long_threshold"), "span_us": round(span, 1),
           "slot_us": round(512 * span), "busy_slot_us": {}}
    for kd, name in ((2, "inter"), (3, "intra")):
        m = ok & (kind == kd)
        out["busy_slot_us"][name] = {"entries": int(m.sum()), "sum_us": round(float((we[m] - ws[m]).sum()))}
    bk = (b[:, 3] >> 32).astype(int)
    okb = b[:, 1] > 0
    bs = (b[:, 0].astype(np.int64) - T0) / 100.0
    be = (b[:, 1].astype(np.int64) - T0) / 100.0
    inter_lens = z["lens"][int(z["n_long"]):]
    width = np.array([inter_lens[i * 64] for i in range(nb)])
    forms = {}
    for kd, name in ((4, "quads"), (3, "tris"), (1, "pairs"), (0, "single")):
        m = okb & (bk == kd)
        if m.any():
            forms[name] = {"blocks": int(m.sum()), "width_min_max": [int(width[m].min()), int(width[m].max())],
                           "dur_us_p0_50_90_100": [round(float(x), 1) for x in
                                                   np.percentile(be[m] - bs[m], [0, 50, 90, 100])],
                           "end_max_us": round(float(be[m].max()), 1)}
    out["inter_forms"] = forms
    m = ok & (kind == 3)
    out["intra_start_us_p0_10_50_90_100"] = [round(float(x), 1) for x in np.percentile(ws[m], [0, 10, 50, 90, 100])]
    out["intra_dur_us_p0_50_90_100"] = [round(float(x), 1) for x in np.percentile(we[m] - ws[m], [0, 50, 90, 100])]
    xs = np.linspace(0, span, 21)
    out["inflight_every_5pct"] = [int(((ws[ok] <= x) & (we[ok] > x)).sum()) for x in xs]
    idx = np.nonzero(ok)[0][np.argsort(-we[ok])]
    out["last_to_end"] = [{"entry": int(k), "kind": "inter" if kind[k] == 2 else "intra",
                           "start_us": round(float(ws[k]), 1), "end_us": round(float(we[k]), 1)} for k in idx[:8]]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
