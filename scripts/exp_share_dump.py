"""Raw block timeline of one rank's share of the strong-scaled C2 database,
for offline analysis (run with a -DSW_TRACE_BLOCKS build via SW_AMD_LIB and
SW_TRACE_FILE set).  Writes OUT.npz: trace [entries][start, end, HW_ID,
XCC_ID | kind << 32] (s_memrealtime, 100 MHz), the block widths, the long
subjects' lengths and the library's timing of the traced scan.
usage: exp_share_dump.py SHARD_OF[:RANK] OUT.npz [LONG_THRESHOLD] [ref]
(ref: the reference's scoring, BLOSUM50 with linear gap 2; default BLOSUM62
affine 11/1)"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import _swpkg  # noqa: E402

sw = _swpkg.load()
path = os.environ["SW_TRACE_FILE"]
S, R = (int(x) for x in (sys.argv[1] + ":0").split(":")[:2])
out = sys.argv[2]
T = int(sys.argv[3]) if len(sys.argv) > 3 else 0
REF = len(sys.argv) > 4 and sys.argv[4] == "ref"
res, offs = sw.synth.database(570000, shard=0)
if S > 1:
    _, res, offs = sw.dist.shard(res, offs, R, S)
with open(os.path.join(REPO, "tests", "golden", "queries", "P07327.fasta")) as f:
    q = sw.encode("".join(f.read().split("\n")[1:]))
h = sw.Handle(0)
db = sw.Database(h, res, offs, long_threshold=(T or None))
m = sw.builtin_matrix(sw.MATRIX_BLOSUM50_REF if REF else sw.MATRIX_BLOSUM62)
go, ge = (2, 2) if REF else (12, 1)
for _ in range(4):
    db.scan(q, matrix=m, gap_open=go, gap_extend=ge)
st = db.stats()
tm = h.timing()
kernel = h.last_kernel()
db.close()
t = np.fromfile(path, dtype=np.uint64).reshape(-1, 4)
lens = np.sort(offs[1:] - offs[:-1])[::-1]
np.savez_compressed(out, trace=t, lens=lens, n_long=st["n_long"], n_blocks=st["n_blocks"],
                    stats=json.dumps(st), timing=json.dumps(tm), kernel=kernel)
print(json.dumps({"stats": st, "timing": tm, "kernel": kernel}))
