"""Experiment: does the two-strips kernel's LDS profile read pay for bank
conflicts?  Same subject lengths, three residue mixes: Swiss-Prot
frequencies (codes c and c + 16 share a 16-byte LDS slot -> 2-way conflicts
inside a ds_read_b128 lane group), uniform over codes 0..15 (one slot per
code: conflict-free), and a single code (broadcast).  Prints the wave
kernel's ms per scan for each."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import _swpkg  # noqa: E402

sw = _swpkg.load()
from sw_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300000
lens = synth.lengths(n)
offs = np.zeros(n + 1, dtype=np.int64)
offs[1:] = np.cumsum(lens)
tot = int(offs[-1])
rng = np.random.default_rng(7)
mixes = {
    "swissprot": synth.residues(tot),
    "uniform16": rng.integers(0, 16, size=tot, dtype=np.uint8),
    "single": np.zeros(tot, dtype=np.uint8),
}
with open(os.path.join(REPO, "tests", "golden", "queries", "P07327.fasta")) as f:
    q = sw.encode("".join(f.read().split("\n")[1:]))
mat = sw.builtin_matrix(sw.MATRIX_BLOSUM62)
h = sw.Handle(0)
out = {}
for name, res in mixes.items():
    db = sw.Database(h, res, offs, long_threshold=100000)
    for _ in range(2):
        db.scan(q, matrix=mat, gap_open=12, gap_extend=1)
    h.timing_reset()
    for _ in range(5):
        db.scan(q, matrix=mat, gap_open=12, gap_extend=1)
    kt = h.timing_total()
    out[name] = {"wave_ms": kt["wave_ms"] / kt["scans"], "kernel": h.last_kernel(),
                 "gcups": len(q) * tot / (kt["wave_ms"] / kt["scans"] * 1e-3) / 1e9}
    db.close()
print(json.dumps(out))
