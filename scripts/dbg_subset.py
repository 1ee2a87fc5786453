"""Debug: the 111-record subset against P02232 / P01008 under several
library settings; prints mismatches against the golden scores."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import _swpkg
from conftest import GOLDEN, read_golden, read_query
import sw_oracle as oracle
sw = _swpkg.load()
recs = oracle.read_fasta_records(GOLDEN + "/subset111.fasta")
seqs = [s for _, s in recs]
res = np.concatenate([oracle.encode(s) for s in seqs])
offs = np.zeros(len(seqs) + 1, dtype=np.int64)
offs[1:] = np.cumsum([len(s) for s in seqs])
lens = offs[1:] - offs[:-1]
h = sw.Handle(0)
for qname in ("P02232", "P01008"):
    q = sw.encode(read_query(qname))
    want = np.array(read_golden(qname + ".subset111.scores"), dtype=np.int32)
    for lt in (None, 300, 1, 100000):
        db = sw.Database(h, res, offs, long_threshold=lt)
        got = db.scan(q)
        bad = np.nonzero(got != want)[0]
        print(qname, "lt", lt, "kernel", h.last_kernel(), h.last_intra_kernel(), "bad", len(bad),
              [(int(i), int(lens[i]), int(got[i]), int(want[i])) for i in bad[:8]], flush=True)
        db.close()
