"""CPU: the oracle itself, pinned to the reference's own golden data."""
import json

import numpy as np
import pytest

from conftest import GOLDEN, path_score, read_golden, read_query


def subset(oracle):
    recs = oracle.read_fasta_records(GOLDEN + "/subset111.fasta")
    seqs = [s for _, s in recs]
    res = np.concatenate([oracle.encode(s) for s in seqs])
    offs = np.zeros(len(seqs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(s) for s in seqs])
    return res, offs


@pytest.mark.parametrize("qname", ["P01008", "P02232"])
def test_oracle_matches_reference_golden(oracle, qname):
    """test/reference/<q>.txt lines 0..110 = the 111 records of uniprot_subset.dat."""
    res, offs = subset(oracle)
    got = oracle.scan(oracle.encode(read_query(qname)), res, offs)
    assert got.tolist() == read_golden(qname + ".subset111.scores")


def test_golden_full_files_consistent():
    """The full golden files: 559,228 scores; their first 111 are the subset
    fixtures; maxima are the self-hits."""
    import gzip
    for q, mx in (("P01008", 3037), ("P02232", 910)):
        with gzip.open(GOLDEN + "/%s.full.txt.gz" % q, "rt") as f:
            vals = [int(x) for x in f.read().split()]
        assert len(vals) == 559228
        assert vals[:111] == read_golden(q + ".subset111.scores")
        assert max(vals) == mx


def test_oracle_matches_cpu_cpp(oracle):
    """Maxima printed by the reference's own cpu.cpp (oracle/_ref/cpu_ref)."""
    pairs = json.load(open(GOLDEN + "/cpu_pairs.json"))["pairs"]
    assert len(pairs) >= 40
    for p in pairs:
        assert oracle.score_raw_identity(p["a"], p["b"]) == p["max"], p
        # the same scheme through the encoded path + identity matrix
        m = oracle.matrix(oracle.MATRIX_IDENTITY3)
        assert oracle.score(oracle.encode(p["a"]), oracle.encode(p["b"]), m) == p["max"]


def _render(a, b, al):
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


def test_traceback_matches_cpu_cpp(oracle):
    """Traceback tie rules of cpu.cpp:47-70 reproduce its printed alignments."""
    pairs = json.load(open(GOLDEN + "/cpu_pairs.json"))["pairs"]
    m = oracle.matrix(oracle.MATRIX_IDENTITY3)
    for p in pairs:
        al = oracle.align(oracle.encode(p["a"]), oracle.encode(p["b"]), m)
        assert al["score"] == p["max"]
        assert _render(p["a"], p["b"], al) == (p["aln_a"], p["aln_b"]), p


def test_python_restatement_agrees(oracle):
    rng = np.random.default_rng(5)
    for mid in (0, 1, 2):
        mat = oracle.matrix(mid)
        for _ in range(20):
            q = rng.integers(0, 25, size=rng.integers(1, 40)).astype(np.uint8)
            s = rng.integers(0, 25, size=rng.integers(1, 40)).astype(np.uint8)
            assert oracle.score(q, s, mat) == oracle.score_linear_py(q, s, mat, 2)


def test_affine_reduces_to_linear(oracle):
    """Gotoh with open == extend == g is the reference's linear gap g."""
    rng = np.random.default_rng(6)
    m = oracle.matrix()
    for _ in range(30):
        q = rng.integers(0, 25, size=rng.integers(1, 60)).astype(np.uint8)
        s = rng.integers(0, 25, size=rng.integers(1, 60)).astype(np.uint8)
        for g in (1, 2, 5):
            assert oracle.score(q, s, m, g, g) == oracle.score(q, s, m, g, g, force_affine=True)


def test_affine_traceback(oracle):
    """The affine traceback (swo_align_affine, this build's tie order): its
    score is Gotoh's (swo_score_affine), its path scores exactly that under
    open / extend, and with open == extend it is the linear traceback of
    cpu.cpp's rules, alignment for alignment."""
    rng = np.random.default_rng(8)
    m = oracle.matrix(oracle.MATRIX_BLOSUM62)
    for _ in range(40):
        q = rng.integers(0, 25, size=rng.integers(1, 80)).astype(np.uint8)
        s = rng.integers(0, 25, size=rng.integers(1, 80)).astype(np.uint8)
        if rng.random() < 0.5:  # a planted copy with indels: long gaps worth opening
            s = np.concatenate([s[:10], q[5:30], s[10:14], q[34:60]]).astype(np.uint8)
        for go, ge in ((12, 1), (11, 2), (5, 5)):
            al = oracle.align(q, s, m, go, ge)
            assert al["score"] == oracle.score(q, s, m, go, ge)
            if al["score"] > 0:
                assert path_score(q, s, m, go, ge, al) == al["score"]
                assert al["ops"][0] == "M" and al["ops"][-1] == "M"
        for g in (1, 2, 5):
            # force the affine routine with open == extend through the C entry
            assert oracle.align(q, s, m, g, g) == _affine_equal(oracle, q, s, m, g)


def _affine_equal(oracle, q, s, m, g):
    import ctypes
    q8 = np.ascontiguousarray(q, dtype=np.uint8)
    s8 = np.ascontiguousarray(s, dtype=np.uint8)
    mm = np.ascontiguousarray(m, dtype=np.int8)
    ints = [ctypes.c_int() for _ in range(5)]
    cap = len(q) + len(s) + 1
    buf = ctypes.create_string_buffer(cap)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    best = oracle.lib().swo_align_affine(q8.ctypes.data_as(u8p), len(q8), s8.ctypes.data_as(u8p), len(s8),
                                         mm.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)), g, g,
                                         *[ctypes.byref(x) for x in ints[:4]], buf, cap, ctypes.byref(ints[4]))
    return {"score": best, "q_end": ints[0].value, "s_end": ints[1].value,
            "q_begin": ints[2].value, "s_begin": ints[3].value, "ops": buf.raw[: ints[4].value].decode()}


def test_matrices(oracle):
    b50 = oracle.matrix(0)
    assert (b50 == b50.T).all() and b50.max() == 15 and b50.min() == -5
    assert (b50[24] == 0).all() and (b50[:, 24] == 0).all()   # SWSolver.cu:80
    assert (b50[23, :24] == -1).all()                          # X row
    b62 = oracle.matrix(1)
    assert (b62 == b62.T).all() and b62[17, 17] == 11


def test_char_compat_matrix(oracle):
    """the _char path's table read through its range-ordered
    lookup (SWSolver_char.cu:22-49, :106-179): BLOSUM50 letters, '*' = -5
    against a letter and +1 against itself; the table's L->W typo (+2) is never
    read (L-W and W-L both come out -2)."""
    t = oracle.char_table()
    L, W = oracle.CHAR_ORDER.index("L"), oracle.CHAR_ORDER.index("W")
    assert t[L, W] == 2 and t[W, L] == -2
    m = oracle.matrix(oracle.MATRIX_BLOSUM50_CHAR)
    b50 = oracle.matrix(0)
    cl, cw = oracle.CODE_ORDER.index("L"), oracle.CODE_ORDER.index("W")
    assert m[cl, cw] == m[cw, cl] == -2
    assert (m == m.T).all()
    assert (m[:24, :24] == b50[:24, :24]).all()
    assert (m[24, :24] == -5).all() and (m[:24, 24] == -5).all() and m[24, 24] == 1
    # a few lookups straight on ASCII (query, subject), both orders
    for a, b in [("A", "A"), ("A", "W"), ("P", "Z"), ("Y", "*"), ("*", "*"), ("N", "T"), ("V", "I")]:
        x = oracle.char_lookup(ord(a), ord(b), t)
        y = oracle.char_lookup(ord(b), ord(a), t)
        assert x == y == m[oracle.CODE_ORDER.index(a), oracle.CODE_ORDER.index(b)]


def test_encoding(oracle):
    codes = oracle.encode("ARNDCQEGHILKMFPSTWYVBJZX")
    assert codes.tolist() == list(range(24))
    assert oracle.encode("UOarnd/\r*").tolist() == [24] * 9   # SWSolver.cu:119


def test_edge_cases(oracle):
    m = oracle.matrix()
    e = np.zeros(0, np.uint8)
    assert oracle.score(e, oracle.encode("AAA"), m) == 0
    assert oracle.score(oracle.encode("W"), oracle.encode("W"), m) == 15
    out = oracle.scan(oracle.encode("WW"), e, np.zeros(3, np.int64))
    assert out.tolist() == [0, 0]
