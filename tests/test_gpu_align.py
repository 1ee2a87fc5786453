"""GPU traceback (sw_align) against the alignments the
reference's own cpu.cpp printed (tests/golden/cpu_pairs.json, cpu.cpp:47-108)
and against the oracle's traceback on a scan's top hits; affine gaps against
the oracle's affine traceback (parity unpinned against the reference, which
has none) and against the score of the path itself."""
import json

import numpy as np
import pytest

from conftest import GOLDEN, path_score

pytestmark = pytest.mark.gpu


def render(a, b, al):
    """Alignment rows as cpu.cpp prints them (cpu.cpp:80-108)."""
    i, j = al["q_begin"] - 1, al["s_begin"] - 1
    ra, rb = [], []
    for op in al["ops"]:
        if op == "M":
            ra.append(a[i]); rb.append(b[j]); i += 1; j += 1
        elif op == "I":
            ra.append(a[i]); rb.append("-"); i += 1
        else:
            ra.append("-"); rb.append(b[j]); j += 1
    return "".join(ra), "".join(rb)


def test_align_matches_cpu_cpp_printed_alignments(sw, oracle, handle):
    pairs = json.load(open(GOLDEN + "/cpu_pairs.json"))["pairs"]
    m = sw.capi.builtin_matrix(sw.capi.MATRIX_IDENTITY3)
    subs = [sw.encode(p["b"]) for p in pairs]
    res = np.concatenate(subs)
    offs = np.zeros(len(subs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(x) for x in subs])
    db = sw.Database(handle, res, offs)
    for k, p in enumerate(pairs):
        al = db.align(sw.encode(p["a"]), [k], m)[0]
        assert al["score"] == p["max"], p
        assert render(p["a"], p["b"], al) == (p["aln_a"], p["aln_b"]), (p, al)


@pytest.mark.parametrize("mid,qlen", [(0, 200), (1, 375), (0, 1100)])
def test_align_top_hits_vs_oracle(sw, oracle, handle, mid, qlen):
    r, o = sw.synth.database(400, shard=mid * 7 + qlen)
    q = sw.synth.query(qlen, shard=qlen)
    m = sw.capi.builtin_matrix(mid)
    db = sw.Database(handle, r, o)
    scores = db.scan(q, m, 2, 2)
    ids, _ = sw.capi.topk(scores, 25)
    ids = list(ids) + [0, 399]
    got = db.align(q, ids, m, 2)
    for i, al in zip(ids, got):
        s = r[o[i]:o[i + 1]]
        want = oracle.align(q, s, m, 2)
        assert al == want, (i, al, want)
        assert al["score"] == scores[i]


def test_align_edges(sw, oracle, handle):
    subs = [sw.encode("ACDEFGHIKL"), np.zeros(0, np.uint8), sw.encode("W")]
    res = np.concatenate(subs)
    offs = np.array([0, 10, 10, 11], dtype=np.int64)
    db = sw.Database(handle, res, offs, ids=np.array([5, 9, 2], dtype=np.int32))
    q = sw.encode("DEFG")
    al = db.align(q, [5, 9, 2])
    assert al[0]["score"] > 0 and al[0]["ops"] == "MMMM" and (al[0]["s_begin"], al[0]["s_end"]) == (3, 6)
    assert al[1] == {"score": 0, "q_begin": 0, "q_end": 0, "s_begin": 0, "s_end": 0, "ops": ""}
    assert al[2] == oracle.align(q, subs[2])
    with pytest.raises(sw.capi.SWError):
        db.align(q, [7])  # not an id of this database
    aff = db.align(q, [5, 9, 2], gap=12, gap_extend=1)
    assert aff[0]["ops"] == "MMMM" and aff[1]["score"] == 0
    assert aff[2] == oracle.align(q, subs[2], None, 12, 1)


@pytest.mark.parametrize("mid,qlen,go,ge", [(1, 375, 12, 1), (0, 200, 11, 2), (1, 700, 8, 3)])
def test_align_affine_vs_oracle(sw, oracle, handle, mid, qlen, go, ge):
    """Affine traceback on a scan's top hits and on planted copies of the
    query with insertions and deletions (runs of gap extension): equal to the
    oracle's alignment, its score to the scan's, and its path scores that."""
    rng = np.random.default_rng(qlen + go)
    r, o = sw.synth.database(300, shard=qlen + 11)
    q = sw.synth.query(qlen, shard=qlen + 3)
    subs = [r[o[i]:o[i + 1]] for i in range(300)]
    for k in range(4):  # query pieces with gaps of 1-9 residues cut out / put in
        a, b = sorted(rng.integers(20, qlen - 20, size=2))
        ins = rng.integers(0, 20, size=int(rng.integers(1, 10))).astype(np.uint8)
        subs[50 * k + 7] = np.concatenate([q[:a], q[a + int(rng.integers(1, 10)):b], ins, q[b:]]).astype(np.uint8)
    res = np.concatenate(subs)
    offs = np.zeros(301, dtype=np.int64)
    offs[1:] = np.cumsum([len(x) for x in subs])
    m = sw.capi.builtin_matrix(mid)
    db = sw.Database(handle, res, offs)
    scores = db.scan(q, m, go, ge)
    ids, _ = sw.capi.topk(scores, 20)
    ids = sorted(set(int(i) for i in ids) | {7, 57, 107, 157, 0, 299})
    got = db.align(q, ids, m, go, ge)
    mm = oracle.matrix(mid)
    for i, al in zip(ids, got):
        want = oracle.align(q, subs[i], mm, go, ge)
        assert al == want, (i, al, want)
        assert al["score"] == scores[i]
        if al["score"] > 0:
            assert path_score(q, subs[i], mm, go, ge, al) == al["score"]
    assert any("DD" in al["ops"] or "II" in al["ops"] for al in got), "a gap run extends"
