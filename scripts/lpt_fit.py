"""The merged launch's duration estimates (csrc/sw_plan.cpp lpt_plan) against
a -DSW_TRACE_BLOCKS timeline of the same scan (exp_share_dump.py .npz): per
item form (quad / tri groups, pairs, single-wave workgroups, tail pairs,
intra workgroups, pipelined pairs) the ratio of the measured duration to the
estimate, by table position, and where the launch's last items sit.
Builds scripts/plan_dump.cpp against sw_plan.cpp (hipcc) on first use.
usage: lpt_fit.py TRACE.npz NPAIR NQUAD NTAIL ROWS RI [TRI=0] [QLEN=375]"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "ece1782-smith-waterman-cuda_amd", "csrc")


def plan_dump_exe():
    exe = os.path.join(tempfile.gettempdir(), "sw_plan_dump")
    srcs = [os.path.join(REPO, "scripts", "plan_dump.cpp"), os.path.join(CSRC, "sw_plan.cpp")]
    if not os.path.exists(exe) or any(os.path.getmtime(s) > os.path.getmtime(exe) for s in srcs):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O1", "-std=c++17", "-I" + CSRC,
                        "-I" + os.path.join(REPO, "include")] + srcs + ["-o", exe], check=True)
    return exe


def main():
    path = sys.argv[1]
    npair, nquad, ntail, rows, ri = (int(x) for x in sys.argv[2:7])
    tri = len(sys.argv) > 7 and sys.argv[7] == "1"
    qlen = int(sys.argv[8]) if len(sys.argv) > 8 else 375
    z = np.load(path)
    kernel = str(z["kernel"])
    affine = "affine" in kernel
    lens = z["lens"]
    nlong = int(z["n_long"])
    order = np.argsort(-lens, kind="stable")
    sl = lens[order]
    llen = sl[:nlong].astype(np.int32)
    short = sl[nlong:]
    nb = int(z["n_blocks"])
    groups = ((short[::64][:nb] + 15) // 16).astype(np.uint32)
    qpad = -(-qlen // rows) * rows
    qpad_intra = -(-qlen // (64 * ri)) * (64 * ri)
    with tempfile.TemporaryDirectory() as d:
        groups.tofile(os.path.join(d, "g"))
        llen.tofile(os.path.join(d, "l"))
        out = subprocess.run([plan_dump_exe(), os.path.join(d, "g"), os.path.join(d, "l"), str(len(lens)),
                              str(int(lens.sum())), str(qpad), str(rows), str(qpad_intra), str(ri), str(npair),
                              str(nquad), str(ntail), str(int(affine)), str(int(tri)), os.path.join(d, "o")],
                             check=True, capture_output=True, text=True).stdout.split()
        npipe, pipe_tail = int(out[0]), int(out[1])
        item = np.fromfile(os.path.join(d, "o.order"), dtype=np.int32)
        cost = np.fromfile(os.path.join(d, "o.cost"), dtype=np.float32)
    t = z["trace"]
    b, w = t[:nb], t[nb:nb + len(item)]
    T0 = b[b[:, 1] > 0, 0].astype(np.int64).min()
    ws = (w[:, 0].astype(np.int64) - T0) / 100.0
    we = (w[:, 1].astype(np.int64) - T0) / 100.0
    dur = we - ws
    pwg = nquad + (npair - nquad + 1) // 2
    tail = nb - ntail
    nspare = max(0, min(nquad, tail - npair)) if tri else 0
    swg = -(-(tail - npair - nspare) // 4)
    npairs = (nlong + 1) // 2
    iwg = -(-npairs // 4)
    form = np.empty(len(item), dtype=object)
    for k, it in enumerate(item):
        if it >= 0:
            form[k] = ("tri" if tri else "quad") if it < nquad else "pair" if it < pwg else "single" \
                if it < pwg + swg else "tailpair"
        else:
            form[k] = "intra" if -1 - it < iwg else "pipe"
    span = float(we.max())
    res = {"kernel": kernel, "entries": int(len(item)), "span_us": round(span, 1), "npipe": npipe,
           "pipe_tail": pipe_tail, "forms": {}}
    ratio = dur / np.maximum(cost, 1e-3)
    for f in ("quad", "tri", "pair", "single", "tailpair", "intra", "pipe"):
        m = form == f
        if not m.any():
            continue
        r = ratio[m & (cost < 1e29)]
        res["forms"][f] = {"entries": int(m.sum()), "first_last_pos": [int(np.nonzero(m)[0][0]),
                                                                    int(np.nonzero(m)[0][-1])],
                           "ratio_p10_50_90": [round(float(x), 3) for x in np.percentile(r, [10, 50, 90])]
                           if len(r) else None,
                           "dur_us_p50_max": [round(float(np.median(dur[m])), 1), round(float(dur[m].max()), 1)]}
    # the items ending in the last 5 % of the span: form, position, start, duration, estimate
    late = np.nonzero(we > 0.95 * span)[0]
    res["late_by_form"] = {f: int((form[late] == f).sum()) for f in set(form[late])}
    res["last_to_end"] = [{"pos": int(k), "form": form[k], "start_us": round(float(ws[k]), 1),
                           "dur_us": round(float(dur[k]), 1), "est_us": round(float(cost[k]), 1)}
                          for k in np.argsort(-we)[:10]]
    # measured duration against table position (deciles)
    dec = np.array_split(np.arange(len(item)), 10)
    res["dur_us_by_decile_p50_max"] = [[round(float(np.median(dur[i])), 1), round(float(dur[i].max()), 1)]
                                       for i in dec]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
