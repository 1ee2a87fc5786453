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
        _LIB = L
    return _LIB


def _u8(a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def matrix(mid=MATRIX_BLOSUM50_REF):
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


def align(q, s, mat=None, gap=2):
    """Score + traceback under cpu.cpp's tie rules. Returns dict."""
    mat = matrix() if mat is None else mat
    q, qp = _u8(q)
    s, sp = _u8(s)
    m, mp = _mat_ptr(mat)
    ints = [ctypes.c_int() for _ in range(5)]
    cap = len(q) + len(s) + 1
    buf = ctypes.create_string_buffer(cap)
    best = lib().swo_align_linear(qp, len(q), sp, len(s), mp, gap,
                                  *[ctypes.byref(x) for x in ints[:4]], buf, cap,
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
