"""Python face of the CPU oracle (oracle/liboracle.so, built from sw_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker / the timed CPU baseline.  The
product path (the HIP library and its C++/Python hosts) never imports this.

Also holds a pure-Python restatement (`score_linear_py`) of the recurrence
for tiny cases, so the C oracle is itself cross-checked.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

MATRIX_BLOSUM50_REF = 0   # SWSolver.cu:54-81
MATRIX_BLOSUM62 = 1       # option, unpinned
MATRIX_IDENTITY3 = 2      # cpu.cpp:6-8


def build():
    """Compile liboracle.so (gcc).  Cheap; called by __graft_entry__.build()."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    if os.path.isdir("/root/reference/src"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.swo_matrix.restype = ctypes.POINTER(ctypes.c_int8)
        L.swo_matrix.argtypes = [ctypes.c_int]
        L.swo_encode.restype = ctypes.c_int64
        L.swo_encode.argtypes = [ctypes.c_char_p, ctypes.c_int64, u8p]
        L.swo_score_linear.restype = ctypes.c_int
        L.swo_score_linear.argtypes = [u8p, ctypes.c_int, u8p, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_int8), ctypes.c_int]
        L.swo_score_affine.restype = ctypes.c_int
        L.swo_score_affine.argtypes = [u8p, ctypes.c_int, u8p, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_int8), ctypes.c_int, ctypes.c_int]
        L.swo_score_raw_identity.restype = ctypes.c_int
        L.swo_score_raw_identity.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.swo_scan.restype = None
        L.swo_scan.argtypes = [u8p, ctypes.c_int, u8p, ctypes.POINTER(ctypes.c_int64),
                               ctypes.c_int64, ctypes.POINTER(ctypes.c_int8), ctypes.c_int,
                               ctypes.c_int, ctypes.POINTER(ctypes.c_int32), ctypes.c_int]
        L.swo_align_linear.restype = ctypes.c_int
        L.swo_align_linear.argtypes = [u8p, ctypes.c_int, u8p, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_int8), ctypes.c_int] + \
            [ctypes.POINTER(ctypes.c_int)] * 4 + [ctypes.c_char_p, ctypes.c_int,
                                                  ctypes.POINTER(ctypes.c_int)]
        L.swo_align_affine.restype = ctypes.c_int
        L.swo_align_affine.argtypes = [u8p, ctypes.c_int, u8p, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_int8), ctypes.c_int, ctypes.c_int] + \
            [ctypes.POINTER(ctypes.c_int)] * 4 + [ctypes.c_char_p, ctypes.c_int,
                                                  ctypes.POINTER(ctypes.c_int)]
        _LIB = L
    return _LIB


def _u8(a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


MATRIX_BLOSUM50_CHAR = 3  # SWSolver_char.cu:22-49 through its lookup :106-179

CODE_ORDER = "ARNDCQEGHILKMFPSTWYVBJZX*"   # SWSolver.cu:17-41
CHAR_ORDER = "ABCDEFGHIJKLMNPQRSTVWXYZ*"   # SWSolver_char.cu:23 (alphabetical, no O/U)


def char_table():
    """The char path's 25x25 table in its alphabetical order
    (SWSolver_char.cu:22-49).  Its letter entries are the reference BLOSUM50's
    (SWSolver.cu:54-81; checked entry by entry against the source), except the
    typo L->W = +2 (:35, W->L is -2 at :44); '*' rows/columns are -5 and
    '*'/'*' is +1 (:48)."""
    ref = matrix(MATRIX_BLOSUM50_REF)
    t = np.zeros((25, 25), dtype=np.int64)
    for i, a in enumerate(CHAR_ORDER):
        for j, b in enumerate(CHAR_ORDER):
            if a == "*" or b == "*":
                t[i, j] = 1 if a == b else -5
            else:
                t[i, j] = ref[CODE_ORDER.index(a), CODE_ORDER.index(b)]
    t[CHAR_ORDER.index("L"), CHAR_ORDER.index("W")] = 2
    return t


def char_lookup(query, subject, t):
    """f_scoreSequence's substitution lookup on ASCII values
    (SWSolver_char.cu:106-179), restated branch by branch: the pair is ordered
    by alphabet range (A-N < P-T < V-Z,'*'), the query first within a range,
    and the flat 625-entry table indexed with the range's ASCII offset
    (65 / 66 / 67: the alphabet without O and U)."""
    q, s = query, subject
    flat = t.reshape(625)

    def vstar(c):
        return c > 85 or c == 42

    if vstar(q) and vstar(s):
        if q == 42 and s == 42:
            return 1
        if q == 42 or s == 42:
            return -5
        return int(flat[(q - 67) * 25 + s - 67])
    if vstar(q) and s > 79:
        return -5 if q == 42 else int(flat[(q - 67) * 25 + s - 66])
    if q > 79 and vstar(s):
        q, s = s, q
        return -5 if q == 42 else int(flat[(q - 67) * 25 + s - 66])
    if vstar(q):
        return -5 if q == 42 else int(flat[(q - 67) * 25 + s - 65])
    if vstar(s):
        q, s = s, q
        return -5 if q == 42 else int(flat[(q - 67) * 25 + s - 65])
    if q > 79 and s > 79:
        return int(flat[(q - 66) * 25 + s - 66])
    if q > 79:
        return int(flat[(q - 66) * 25 + s - 65])
    if s > 79:
        q, s = s, q
        return int(flat[(q - 66) * 25 + s - 65])
    return int(flat[(q - 65) * 25 + s - 65])


def char_compat_matrix():
    """The char path's effective scores in code order: M[qc][sc] =
    char_lookup(letter(qc), letter(sc)); code 24 is '*', which
    convertStringToChar (SWSolver_char.cu:56-85) also makes of U, O,
    lowercase and the parser's '/' padding."""
    t = char_table()
    m = np.zeros((25, 25), dtype=np.int8)
    for i, a in enumerate(CODE_ORDER):
        for j, b in enumerate(CODE_ORDER):
            m[i, j] = char_lookup(ord(a), ord(b), t)
    return m


def matrix(mid=MATRIX_BLOSUM50_REF):
    if mid == MATRIX_BLOSUM50_CHAR:
        return char_compat_matrix()
    p = lib().swo_matrix(mid)
    return np.ctypeslib.as_array(p, shape=(625,)).copy().reshape(25, 25)


def _mat_ptr(mat):
    m = np.ascontiguousarray(np.asarray(mat, dtype=np.int8).reshape(625))
    return m, m.ctypes.data_as(ctypes.POINTER(ctypes.c_int8))


def encode(seq):
    """ASCII -> codes 0..24 (SWSolver.cu:91-120)."""
    b = seq.encode() if isinstance(seq, str) else bytes(seq)
    out = np.empty(len(b), dtype=np.uint8)
    lib().swo_encode(b, len(b), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    return out


def score(q, s, mat=None, gap_open=2, gap_extend=2, force_affine=False):
    """One pair, encoded inputs (go == ge uses the linear recurrence unless
    force_affine)."""
    mat = matrix() if mat is None else mat
    q, qp = _u8(q)
    s, sp = _u8(s)
    m, mp = _mat_ptr(mat)
    if gap_open == gap_extend and not force_affine:
        return lib().swo_score_linear(qp, len(q), sp, len(s), mp, gap_open)
    return lib().swo_score_affine(qp, len(q), sp, len(s), mp, gap_open, gap_extend)


def score_raw_identity(a, b, match=3, mismatch=-3, gap=2):
    """cpu.cpp on raw strings."""
    ab, bb = a.encode(), b.encode()
    return lib().swo_score_raw_identity(ab, len(ab), bb, len(bb), match, mismatch, gap)


def scan(q, residues, offsets, mat=None, gap_open=2, gap_extend=2, nthreads=0):
    """Score encoded query q against subjects residues[offsets[k]:offsets[k+1]]."""
    mat = matrix() if mat is None else mat
    q, qp = _u8(q)
    r, rp = _u8(residues)
    o = np.ascontiguousarray(offsets, dtype=np.int64)
    n = len(o) - 1
    out = np.zeros(max(n, 0), dtype=np.int32)
    m, mp = _mat_ptr(mat)
    if n > 0:
        lib().swo_scan(qp, len(q), rp, o.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), n, mp,
                       gap_open, gap_extend, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                       int(nthreads))
    return out


def align(q, s, mat=None, gap=2, gap_extend=None):
    """Score + traceback under cpu.cpp's tie rules (oracle/sw_oracle.c
    swo_align_linear, cpu.cpp:47-108); with gap_extend != gap the affine
    traceback swo_align_affine (this build's tie order).  Returns dict."""
    mat = matrix() if mat is None else mat
    q, qp = _u8(q)
    s, sp = _u8(s)
    m, mp = _mat_ptr(mat)
    ints = [ctypes.c_int() for _ in range(5)]
    cap = len(q) + len(s) + 1
    buf = ctypes.create_string_buffer(cap)
    refs = [ctypes.byref(x) for x in ints[:4]]
    if gap_extend is None or gap_extend == gap:
        best = lib().swo_align_linear(qp, len(q), sp, len(s), mp, gap, *refs, buf, cap, ctypes.byref(ints[4]))
    else:
        best = lib().swo_align_affine(qp, len(q), sp, len(s), mp, gap, gap_extend, *refs, buf, cap,
                                      ctypes.byref(ints[4]))
    return {"score": best, "q_end": ints[0].value, "s_end": ints[1].value,
            "q_begin": ints[2].value, "s_begin": ints[3].value,
            "ops": buf.raw[: ints[4].value].decode()}


def score_linear_py(q, s, mat, gap):
    """Pure-Python restatement of SWSolver.cu:246 for tiny cases."""
    best = 0
    prev = [0] * (len(s) + 1)
    for i in range(1, len(q) + 1):
        cur = [0] * (len(s) + 1)
        for j in range(1, len(s) + 1):
            h = max(0, prev[j - 1] + int(mat[q[i - 1]][s[j - 1]]), cur[j - 1] - gap, prev[j] - gap)
            cur[j] = h
            best = max(best, h)
        prev = cur
    return best


def read_fasta_records(path):
    """(header, sequence) records; sequence lines concatenated verbatim."""
    recs, head, seq = [], None, []
    with open(path) as f:
        for line in f:
            line = line.rstrip("\n")
            if line.startswith(">"):
                if head is not None:
                    recs.append((head, "".join(seq)))
                head, seq = line, []
            else:
                seq.append(line)
    if head is not None:
        recs.append((head, "".join(seq)))
    return recs
