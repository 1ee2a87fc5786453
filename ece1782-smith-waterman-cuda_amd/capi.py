"""ctypes binding of the C ABI in include/sw_amd.h (lib/libswamd.so).

This is the product path's Python face: it loads ONLY the in-tree HIP
library and raises if it is missing — there is no CPU fallback.
"""
import ctypes
import os
import weakref

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(PKG_DIR, "lib")
# SW_AMD_LIB: an alternative build of the same library (A/B kernel experiments)
LIB_PATH = os.environ.get("SW_AMD_LIB") or os.path.join(LIB_DIR, "libswamd.so")

SW_OK = 0
SW_ALPHABET = 25
MATRIX_BLOSUM50_REF = 0
MATRIX_BLOSUM62 = 1
MATRIX_IDENTITY3 = 2
MATRIX_BLOSUM50_CHAR = 3  # the _char path's table as its lookup reads it ('*' = -5)

# Every symbol include/sw_amd.h declares (checked by tests/test_abi.py).
EXPORTED = (
    "sw_version", "sw_build_id", "sw_last_error", "sw_encode", "sw_builtin_matrix",
    "sw_create", "sw_destroy", "sw_stream", "sw_set_stream",
    "sw_opts_init", "sw_opts_from_env", "sw_set_opts", "sw_get_opts",
    "sw_db_create", "sw_db_free", "sw_db_get_stats", "sw_db_set_long_threshold", "sw_db_reset_adaptive",
    "sw_scan", "sw_scan_device", "sw_scan_batch", "sw_scan_batch_device", "sw_get_timing",
    "sw_timing_reset", "sw_timing_total", "sw_stream_wait_scan", "sw_last_kernel", "sw_last_intra_kernel",
    "sw_topk", "sw_topk_device", "sw_topk_keys_device", "sw_topk_device_ids", "sw_scan_topk",
    "sw_scan_rank_device", "sw_score_pair",
    "sw_align",
    "sw_db_save", "sw_db_load", "sw_db_subjects", "sw_db_create_synthetic", "sw_synth_tables",
    "sw_synth_lengths", "sw_group_create", "sw_group_destroy", "sw_group_info", "sw_group_handle",
    "sw_group_db_create", "sw_group_db_free", "sw_group_db_shard", "sw_group_scan", "sw_group_topk",
)


class SWError(RuntimeError):
    pass


class Scoring(ctypes.Structure):
    _fields_ = [("matrix", ctypes.POINTER(ctypes.c_int8)),
                ("gap_open", ctypes.c_int32),
                ("gap_extend", ctypes.c_int32)]


class DbStats(ctypes.Structure):
    _fields_ = [("n_subjects", ctypes.c_int64), ("residues", ctypes.c_int64),
                ("packed_cells", ctypes.c_int64), ("n_blocks", ctypes.c_int64),
                ("n_long", ctypes.c_int64), ("device_bytes", ctypes.c_int64),
                ("max_length", ctypes.c_int32), ("long_threshold", ctypes.c_int32),
                ("coop_blocks", ctypes.c_int32), ("coop_residues", ctypes.c_int64),
                ("max_id", ctypes.c_int32), ("pair_blocks", ctypes.c_int32),
                ("pair_merged", ctypes.c_int32), ("pair_residues", ctypes.c_int64)]


class Alignment(ctypes.Structure):
    _fields_ = [("score", ctypes.c_int32), ("q_begin", ctypes.c_int32), ("q_end", ctypes.c_int32),
                ("s_begin", ctypes.c_int32), ("s_end", ctypes.c_int32), ("ops_len", ctypes.c_int32)]


class Opts(ctypes.Structure):
    """sw_opts (include/sw_amd.h): kernel-form overrides, -1 = the library's
    choice.  Field names are the header's; the SW_* variable each mirrors
    is listed there."""
    INT_FIELDS = ("lpt", "lpt_pipe", "quad_width", "pair_width", "pair_group", "coop_width", "coop_skew",
                  "intra_x2", "intra_x2_rows", "intra_i16_first", "inter_i16_span", "int16_guard",
                  "rescue_stats", "tail_pairs", "lpt_persist", "lpt_rows", "tri_width", "lpt_pipe_tail", "drain_spin")
    _fields_ = [("size", ctypes.c_int32)] + [(f, ctypes.c_int32) for f in INT_FIELDS] + \
        [("inter_variant", ctypes.c_char * 16), ("trace_file", ctypes.c_char * 256)]

    def as_dict(self):
        d = {f: getattr(self, f) for f in self.INT_FIELDS}
        d["inter_variant"] = self.inter_variant.decode()
        d["trace_file"] = self.trace_file.decode()
        return d


def opts_from_env():
    """sw_opts from the SW_* environment (sw_opts_from_env)."""
    o = Opts()
    _check(lib().sw_opts_from_env(ctypes.byref(o)))
    return o


class Timing(ctypes.Structure):
    _fields_ = [("inter_ms", ctypes.c_float), ("intra_ms", ctypes.c_float),
                ("total_ms", ctypes.c_float), ("rescued", ctypes.c_int32),
                ("launches", ctypes.c_int32), ("coop_ms", ctypes.c_float),
                ("wave_ms", ctypes.c_float)]


_LIB = None


def lib():
    """Load lib/libswamd.so (built by build()); raise if absent."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise SWError("HIP library %s not built; run __graft_entry__.build() "
                      "or make -C ece1782-smith-waterman-cuda_amd/csrc" % LIB_PATH)
    # One HIP runtime per process: PyTorch-ROCm bundles its own
    # libamdhip64.so with the same SONAME (libamdhip64.so.7) as /opt/rocm's.
    # Imported first, it is the runtime our library binds to, and streams can
    # be shared; loaded after us it would start a second runtime that cannot
    # see the GPU.  (PyTorch is plumbing here, not a dependency: without it
    # the library uses the system runtime.)
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    u8p = ctypes.POINTER(ctypes.c_uint8)
    i32p = ctypes.POINTER(ctypes.c_int32)
    i64p = ctypes.POINTER(ctypes.c_int64)
    sig = {
        "sw_version": (i32, []),
        "sw_build_id": (ctypes.c_char_p, []),
        "sw_last_error": (ctypes.c_char_p, []),
        "sw_encode": (ctypes.c_int, [ctypes.c_char_p, i64, u8p]),
        "sw_builtin_matrix": (ctypes.c_int, [i32, ctypes.POINTER(ctypes.c_int8)]),
        "sw_create": (ctypes.c_int, [i32, ctypes.POINTER(vp)]),
        "sw_destroy": (ctypes.c_int, [vp]),
        "sw_stream": (vp, [vp]),
        "sw_set_stream": (ctypes.c_int, [vp, vp]),
        "sw_opts_init": (ctypes.c_int, [ctypes.POINTER(Opts)]),
        "sw_opts_from_env": (ctypes.c_int, [ctypes.POINTER(Opts)]),
        "sw_set_opts": (ctypes.c_int, [vp, ctypes.POINTER(Opts)]),
        "sw_get_opts": (ctypes.c_int, [vp, ctypes.POINTER(Opts)]),
        "sw_db_reset_adaptive": (ctypes.c_int, [vp]),
        "sw_db_create": (ctypes.c_int, [vp, u8p, i64p, i64, i32p, ctypes.POINTER(vp)]),
        "sw_db_free": (ctypes.c_int, [vp]),
        "sw_db_get_stats": (ctypes.c_int, [vp, ctypes.POINTER(DbStats)]),
        "sw_db_set_long_threshold": (ctypes.c_int, [vp, i32]),
        "sw_scan": (ctypes.c_int, [vp, vp, u8p, i32, ctypes.POINTER(Scoring), i32p]),
        "sw_scan_device": (ctypes.c_int, [vp, vp, u8p, i32, ctypes.POINTER(Scoring), vp]),
        "sw_scan_batch": (ctypes.c_int, [vp, vp, u8p, i64p, i32, ctypes.POINTER(Scoring), i32p]),
        "sw_scan_batch_device": (ctypes.c_int, [vp, vp, u8p, i64p, i32, ctypes.POINTER(Scoring), vp]),
        "sw_get_timing": (ctypes.c_int, [vp, ctypes.POINTER(Timing)]),
        "sw_timing_reset": (ctypes.c_int, [vp]),
        "sw_timing_total": (ctypes.c_int, [vp, ctypes.POINTER(Timing), i32p]),
        "sw_stream_wait_scan": (ctypes.c_int, [vp, vp]),
        "sw_last_kernel": (ctypes.c_char_p, [vp]),
        "sw_last_intra_kernel": (ctypes.c_char_p, [vp]),
        "sw_db_save": (ctypes.c_int, [vp, ctypes.c_char_p]),
        "sw_db_create_synthetic": (ctypes.c_int, [vp, ctypes.c_uint64, i64, i64, ctypes.POINTER(vp)]),
        "sw_synth_tables": (ctypes.c_int, [i32p, u8p]),
        "sw_synth_lengths": (ctypes.c_int, [ctypes.c_uint64, i64, i64, i32p]),
        "sw_db_subjects": (ctypes.c_int, [vp, i64p, i32p]),
        "sw_db_load": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.POINTER(vp)]),
        "sw_align": (ctypes.c_int, [vp, vp, u8p, i32, ctypes.POINTER(Scoring), i32p, i32,
                                    ctypes.POINTER(Alignment), ctypes.c_char_p, ctypes.c_int64]),
        "sw_topk": (ctypes.c_int, [i32p, i64, i32, i32p, i32p]),
        "sw_topk_device": (ctypes.c_int, [vp, vp, i64, i64, i32, vp]),
        "sw_topk_keys_device": (ctypes.c_int, [vp, vp, i64, i32, vp]),
        "sw_topk_device_ids": (ctypes.c_int, [vp, vp, i64, vp, i32, vp]),
        "sw_scan_topk": (ctypes.c_int, [vp, vp, u8p, i32, ctypes.POINTER(Scoring), i32, i64p]),
        "sw_scan_rank_device": (ctypes.c_int, [vp, vp, u8p, i32, ctypes.POINTER(Scoring), vp, i32, vp, i64, vp]),
        "sw_score_pair": (ctypes.c_int, [vp, u8p, i32, u8p, i32, ctypes.POINTER(Scoring), i32p]),
        "sw_group_create": (ctypes.c_int, [i32p, i32, ctypes.POINTER(vp)]),
        "sw_group_destroy": (ctypes.c_int, [vp]),
        "sw_group_info": (ctypes.c_char_p, [vp]),
        "sw_group_handle": (ctypes.c_int, [vp, i32, ctypes.POINTER(vp)]),
        "sw_group_db_create": (ctypes.c_int, [vp, u8p, i64p, i64, i32p, ctypes.POINTER(vp)]),
        "sw_group_db_free": (ctypes.c_int, [vp]),
        "sw_group_db_shard": (ctypes.c_int, [vp, i32, i64p, i64p]),
        "sw_group_scan": (ctypes.c_int, [vp, vp, u8p, i32, ctypes.POINTER(Scoring), i32p]),
        "sw_group_topk": (ctypes.c_int, [vp, vp, u8p, i32, ctypes.POINTER(Scoring), i32, i64p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    built, want = L.sw_build_id().decode(), source_id()
    if built != want:
        raise SWError("stale HIP library %s: built from sources %s, the tree's are %s; rebuild it "
                      "(__graft_entry__.build() or make -C ece1782-smith-waterman-cuda_amd/csrc)"
                      % (LIB_PATH, built, want))
    _LIB = L
    return L


def source_id(repo_root=None):
    """The id of the library sources in this tree (csrc/build_id.py, the
    same computation the Makefile compiles into sw_build_id)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("_sw_build_id", os.path.join(PKG_DIR, "csrc", "build_id.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.source_id(repo_root or os.path.dirname(PKG_DIR))


def build_id():
    """sw_build_id() of the loaded library."""
    return lib().sw_build_id().decode()


def _check(rc):
    if rc != SW_OK:
        raise SWError("sw_amd error %d: %s" % (rc, lib().sw_last_error().decode(errors="replace")))


def _u8(a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def encode(seq):
    """ASCII -> residue codes (SWSolver.cu:91-120 mapping)."""
    b = seq.encode() if isinstance(seq, str) else bytes(seq)
    out = np.empty(len(b), dtype=np.uint8)
    _check(lib().sw_encode(b, len(b), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
    return out


def builtin_matrix(mid=MATRIX_BLOSUM50_REF):
    out = np.empty(625, dtype=np.int8)
    _check(lib().sw_builtin_matrix(mid, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int8))))
    return out.reshape(25, 25)


class _ScoringArg:
    """Keeps the matrix buffer alive for the duration of a call."""

    def __init__(self, matrix=None, gap_open=2, gap_extend=None):
        gap_extend = gap_open if gap_extend is None else gap_extend
        if matrix is None:
            self._m = None
            self.s = Scoring(None, gap_open, gap_extend)
        else:
            self._m = np.ascontiguousarray(np.asarray(matrix, dtype=np.int8).reshape(625))
            self.s = Scoring(self._m.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)), gap_open, gap_extend)

    def ptr(self):
        return ctypes.byref(self.s)


class Handle:
    """One device + one HIP stream (sw_create).  env_opts: start from the
    SW_* environment (sw_opts_from_env: measurement scripts set kernel-form
    overrides that way); otherwise the library's own choices."""

    def __init__(self, device=0, env_opts=True):
        h = ctypes.c_void_p()
        _check(lib().sw_create(device, ctypes.byref(h)))
        self._h = h
        self.device = device
        self._dbs = weakref.WeakSet()  # databases must be freed before the handle
        if env_opts:
            _check(lib().sw_set_opts(h, ctypes.byref(opts_from_env())))

    def get_opts(self):
        o = Opts()
        _check(lib().sw_get_opts(self._h, ctypes.byref(o)))
        return o

    def set_opts(self, opts=None, **fields):
        """sw_set_opts: `opts` (an Opts; default the handle's current ones)
        with `fields` changed, e.g. set_opts(lpt=1, quad_width=0)."""
        o = Opts()
        if opts is None:
            o = self.get_opts()
        else:
            ctypes.memmove(ctypes.byref(o), ctypes.byref(opts), ctypes.sizeof(Opts))
        for k, v in fields.items():
            if k in ("inter_variant", "trace_file"):
                setattr(o, k, (v or "").encode())
            elif k in Opts.INT_FIELDS:
                setattr(o, k, -1 if v is None else int(v))
            else:
                raise TypeError("unknown sw_opts field %r" % k)
        _check(lib().sw_set_opts(self._h, ctypes.byref(o)))

    def reset_opts(self):
        """Every override off (sw_opts_init: the library's own choices)."""
        o = Opts()
        _check(lib().sw_opts_init(ctypes.byref(o)))
        _check(lib().sw_set_opts(self._h, ctypes.byref(o)))

    @property
    def ptr(self):
        return self._h

    def close(self):
        if self._h:
            for db in list(self._dbs):
                db.close()
            lib().sw_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stream(self):
        return lib().sw_stream(self._h)

    def set_stream(self, hip_stream):
        _check(lib().sw_set_stream(self._h, hip_stream))

    def timing(self):
        t = Timing()
        _check(lib().sw_get_timing(self._h, ctypes.byref(t)))
        return {k: getattr(t, k) for k, _ in Timing._fields_}

    def timing_reset(self):
        _check(lib().sw_timing_reset(self._h))

    def stream_wait_scan(self, hip_stream):
        """Make hip_stream wait for this handle's most recent scan (its end
        event; no event record of the caller's on the scan's stream)."""
        _check(lib().sw_stream_wait_scan(self._h, hip_stream))

    def last_kernel(self):
        """Per-wave inter kernel of the last scan, e.g. 'sw_inter_x2<16,16,affine>'."""
        return lib().sw_last_kernel(self._h).decode()

    def last_intra_kernel(self):
        """Long-subject kernel of the last scan, e.g. 'sw_intra_x2<16>'; 'none'."""
        return lib().sw_last_intra_kernel(self._h).decode()

    def timing_total(self):
        """Kernel ms summed over all scans since timing_reset(); waits."""
        t = Timing()
        n = ctypes.c_int32()
        _check(lib().sw_timing_total(self._h, ctypes.byref(t), ctypes.byref(n)))
        out = {k: getattr(t, k) for k, _ in Timing._fields_ if k != "rescued"}
        out["scans"] = n.value
        return out

    def topk_device(self, scores_dev_ptr, n, k, keys_out_dev_ptr, id_base=0):
        """Asynchronous device top-k into an int64 key buffer (best first)."""
        _check(lib().sw_topk_device(self._h, ctypes.c_void_p(scores_dev_ptr), n, id_base, k,
                                    ctypes.c_void_p(keys_out_dev_ptr)))

    def topk_device_ids(self, scores_dev_ptr, n, ids_dev_ptr, k, keys_out_dev_ptr):
        """Device top-k with global ids from a device int32 id map."""
        _check(lib().sw_topk_device_ids(self._h, ctypes.c_void_p(scores_dev_ptr), n, ctypes.c_void_p(ids_dev_ptr),
                                        k, ctypes.c_void_p(keys_out_dev_ptr)))

    def topk_keys_device(self, keys_dev_ptr, n, k, keys_out_dev_ptr):
        _check(lib().sw_topk_keys_device(self._h, ctypes.c_void_p(keys_dev_ptr), n, k,
                                         ctypes.c_void_p(keys_out_dev_ptr)))

    def score_pair(self, query_codes, subject_codes, matrix=None, gap_open=2, gap_extend=None):
        q, qp = _u8(query_codes)
        s, sp = _u8(subject_codes)
        sc = _ScoringArg(matrix, gap_open, gap_extend)
        out = ctypes.c_int32()
        _check(lib().sw_score_pair(self._h, qp, len(q), sp, len(s), sc.ptr(), ctypes.byref(out)))
        return out.value


class Database:
    """A device-resident packed database (sw_db_create)."""

    def __init__(self, handle, residues, offsets, ids=None, long_threshold=None):
        self.handle = handle
        r, rp = _u8(residues)
        o = np.ascontiguousarray(offsets, dtype=np.int64)
        n = len(o) - 1
        idp = None
        if ids is not None:
            self._ids = np.ascontiguousarray(ids, dtype=np.int32)
            idp = self._ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
            self.n_out = int(self._ids.max()) + 1 if n > 0 else 0
        else:
            self.n_out = n
        d = ctypes.c_void_p()
        _check(lib().sw_db_create(handle.ptr, rp, o.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                  n, idp, ctypes.byref(d)))
        self._d = d
        self.n = n
        handle._dbs.add(self)
        if long_threshold is not None:
            self.set_long_threshold(long_threshold)

    @classmethod
    def synthetic(cls, handle, seed, n, id_base=0, long_threshold=None):
        """A synthetic database generated in HBM (sw_db_create_synthetic):
        subject k (result id k) has global id id_base + k; see synth.counter_*
        for the CPU restatement."""
        self = cls.__new__(cls)
        self.handle = handle
        d = ctypes.c_void_p()
        _check(lib().sw_db_create_synthetic(handle.ptr, seed, id_base, n, ctypes.byref(d)))
        self._d = d
        self.n = n
        self.n_out = n
        handle._dbs.add(self)
        if long_threshold is not None:
            self.set_long_threshold(long_threshold)
        return self

    def subjects(self):
        """(lengths int64[n], ids int32[n]) in database order (sw_db_subjects)."""
        n = self.stats()["n_subjects"]
        L = np.zeros(n, dtype=np.int64)
        ids = np.zeros(n, dtype=np.int32)
        _check(lib().sw_db_subjects(self._d, L.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                    ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return L, ids

    @classmethod
    def load(cls, handle, path, long_threshold=None):
        """A database from a sw_db_save file (one read, no FASTA parsing)."""
        self = cls.__new__(cls)
        self.handle = handle
        d = ctypes.c_void_p()
        _check(lib().sw_db_load(handle.ptr, os.fsencode(path), ctypes.byref(d)))
        self._d = d
        st = self.stats()
        self.n = st["n_subjects"]
        self.n_out = st["max_id"] + 1
        handle._dbs.add(self)
        if long_threshold is not None:
            self.set_long_threshold(long_threshold)
        return self

    def save(self, path):
        """Write the binary database file (sw_db_save)."""
        _check(lib().sw_db_save(self._d, os.fsencode(path)))

    @property
    def ptr(self):
        return self._d

    def close(self):
        if self._d:
            if self.handle.ptr:  # a closed handle already freed us
                lib().sw_db_free(self._d)
            self._d = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_long_threshold(self, t):
        _check(lib().sw_db_set_long_threshold(self._d, int(t)))

    def reset_adaptive(self):
        """Forget the int16-first routing learned from earlier scans
        (sw_db_reset_adaptive): the next scan runs as on a fresh database."""
        _check(lib().sw_db_reset_adaptive(self._d))

    def stats(self):
        s = DbStats()
        _check(lib().sw_db_get_stats(self._d, ctypes.byref(s)))
        return {k: getattr(s, k) for k, _ in DbStats._fields_}

    def scan(self, query_codes, matrix=None, gap_open=2, gap_extend=None):
        """Synchronous scan; returns int32 scores indexed by id."""
        q, qp = _u8(query_codes)
        sc = _ScoringArg(matrix, gap_open, gap_extend)
        out = np.zeros(self.n_out, dtype=np.int32)
        _check(lib().sw_scan(self.handle.ptr, self._d, qp, len(q), sc.ptr(),
                             out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return out

    def scan_device(self, query_codes, scores_dev_ptr, matrix=None, gap_open=2, gap_extend=None):
        """Asynchronous scan on the handle's stream into a device int32 buffer."""
        q, qp = _u8(query_codes)
        sc = _ScoringArg(matrix, gap_open, gap_extend)
        _check(lib().sw_scan_device(self.handle.ptr, self._d, qp, len(q), sc.ptr(),
                                    ctypes.c_void_p(scores_dev_ptr)))

    def scan_rank_device(self, query_codes, scores_dev_ptr, k, keys_out_dev_ptr, matrix=None, gap_open=2,
                         gap_extend=None, gids_dev_ptr=None, id_base=0):
        """Asynchronous scan into a device int32 buffer and the device top-K
        of its scores into keys_out_dev_ptr (k int64 keys, best first, global
        id gids[r] or id_base + r for result id r; sw_scan_rank_device: inside
        the scan's merged launch when it is one)."""
        q, qp = _u8(query_codes)
        sc = _ScoringArg(matrix, gap_open, gap_extend)
        _check(lib().sw_scan_rank_device(self.handle.ptr, self._d, qp, len(q), sc.ptr(),
                                         ctypes.c_void_p(scores_dev_ptr), k, ctypes.c_void_p(gids_dev_ptr or 0),
                                         id_base, ctypes.c_void_p(keys_out_dev_ptr)))

    def scan_topk(self, query_codes, k, matrix=None, gap_open=2, gap_extend=None):
        """The k best subjects as int64 keys (score << 32 | 2^31-1-id, best
        first; sw_scan_topk: scan + device top-K, k keys copied back)."""
        q, qp = _u8(query_codes)
        sc = _ScoringArg(matrix, gap_open, gap_extend)
        out = np.zeros(k, dtype=np.int64)
        _check(lib().sw_scan_topk(self.handle.ptr, self._d, qp, len(q), sc.ptr(), k,
                                  out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        return out

    def align(self, query_codes, ids, matrix=None, gap=2, gap_extend=None):
        """Traceback of the query against the subjects with these result ids
        (sw_align: cpu.cpp's tie rules for a linear gap; gap_extend != gap: the
        affine extension of them, include/sw_amd.h).  Returns a list of dicts
        {score, q_begin, q_end, s_begin, s_end, ops} like the oracle's align."""
        q, qp = _u8(query_codes)
        idv = np.ascontiguousarray(ids, dtype=np.int32)
        n = len(idv)
        sc = _ScoringArg(matrix, gap, gap if gap_extend is None else gap_extend)
        out = (Alignment * max(n, 1))()
        stride = len(q) + int(self.stats()["max_length"]) + 1
        buf = ctypes.create_string_buffer(max(n, 1) * stride)
        _check(lib().sw_align(self.handle.ptr, self._d, qp, len(q), sc.ptr(),
                              idv.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n, out, buf, stride))
        res = []
        for k in range(n):
            a = out[k]
            res.append({"score": a.score, "q_begin": a.q_begin, "q_end": a.q_end, "s_begin": a.s_begin,
                        "s_end": a.s_end, "ops": buf.raw[k * stride: k * stride + a.ops_len].decode()})
        return res

    @staticmethod
    def _cat(queries):
        cat = np.concatenate([np.asarray(q, dtype=np.uint8) for q in queries]) if len(queries) else \
            np.zeros(0, dtype=np.uint8)
        offs = np.zeros(len(queries) + 1, dtype=np.int64)
        offs[1:] = np.cumsum([len(q) for q in queries])
        return cat, offs

    def scan_batch_device(self, queries, scores_dev_ptr, matrix=None, gap_open=2, gap_extend=None):
        """Asynchronous batch scan into a device int32 buffer [nq, n_out]."""
        cat, offs = self._cat(queries)
        c, cp = _u8(cat)
        sc = _ScoringArg(matrix, gap_open, gap_extend)
        _check(lib().sw_scan_batch_device(self.handle.ptr, self._d, cp,
                                          offs.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), len(queries),
                                          sc.ptr(), ctypes.c_void_p(scores_dev_ptr)))

    def scan_batch(self, queries, matrix=None, gap_open=2, gap_extend=None):
        """queries: list of code arrays; returns [nq, n_out] int32."""
        cat, offs = self._cat(queries)
        c, cp = _u8(cat)
        sc = _ScoringArg(matrix, gap_open, gap_extend)
        out = np.zeros((len(queries), self.n_out), dtype=np.int32)
        _check(lib().sw_scan_batch(self.handle.ptr, self._d, cp,
                                   offs.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), len(queries),
                                   sc.ptr(), out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return out


class Group:
    """Several GPUs of this process searching one database (sw_group_*):
    residue-balanced shards, one host thread per device, RCCL all-gather of
    the per-device top-K (a device listed twice: host exchange)."""

    def __init__(self, devices):
        devs = np.ascontiguousarray(devices, dtype=np.int32)
        g = ctypes.c_void_p()
        _check(lib().sw_group_create(devs.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(devs),
                                     ctypes.byref(g)))
        self._g = g
        self.n = len(devs)

    def info(self):
        return lib().sw_group_info(self._g).decode()

    def close(self):
        if self._g:
            lib().sw_group_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def database(self, residues, offsets, ids=None):
        return GroupDatabase(self, residues, offsets, ids)


class GroupDatabase:
    def __init__(self, group, residues, offsets, ids=None):
        self.group = group
        r, rp = _u8(residues)
        o = np.ascontiguousarray(offsets, dtype=np.int64)
        n = len(o) - 1
        idp = None
        self.n_out = n
        if ids is not None:
            self._ids = np.ascontiguousarray(ids, dtype=np.int32)
            idp = self._ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
            self.n_out = int(self._ids.max()) + 1 if n else 0
        d = ctypes.c_void_p()
        _check(lib().sw_group_db_create(group._g, rp, o.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), n, idp,
                                        ctypes.byref(d)))
        self._d = d

    def shard(self, k):
        n, r = ctypes.c_int64(), ctypes.c_int64()
        _check(lib().sw_group_db_shard(self._d, k, ctypes.byref(n), ctypes.byref(r)))
        return n.value, r.value

    def close(self):
        if self._d:
            lib().sw_group_db_free(self._d)
            self._d = None

    def scan(self, query_codes, matrix=None, gap_open=2, gap_extend=None):
        q, qp = _u8(query_codes)
        sc = _ScoringArg(matrix, gap_open, gap_extend)
        out = np.zeros(self.n_out, dtype=np.int32)
        _check(lib().sw_group_scan(self.group._g, self._d, qp, len(q), sc.ptr(),
                                   out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return out

    def topk(self, query_codes, k, matrix=None, gap_open=2, gap_extend=None):
        """int64 keys (score << 32 | 2^31-1-id), best first."""
        q, qp = _u8(query_codes)
        sc = _ScoringArg(matrix, gap_open, gap_extend)
        out = np.zeros(k, dtype=np.int64)
        _check(lib().sw_group_topk(self.group._g, self._d, qp, len(q), sc.ptr(), k,
                                   out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        return out


def synth_tables():
    """(length quantile table int32[4096], u16 -> residue table uint8[65536])
    of the library's synthetic databases."""
    L = np.zeros(4096, dtype=np.int32)
    lut = np.zeros(65536, dtype=np.uint8)
    _check(lib().sw_synth_tables(L.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                 lut.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
    return L, lut


def synth_lengths(seed, id_base, n):
    out = np.zeros(n, dtype=np.int32)
    _check(lib().sw_synth_lengths(seed, id_base, n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
    return out


def topk(scores, k):
    """(ids, scores) of the k best: score descending, id ascending."""
    s = np.ascontiguousarray(scores, dtype=np.int32)
    ids = np.empty(k, dtype=np.int32)
    vals = np.empty(k, dtype=np.int32)
    _check(lib().sw_topk(s.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(s), k,
                         ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                         vals.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
    return ids, vals


def decode_keys(keys):
    """int64 top-k keys -> (ids, scores); INT64_MIN padding -> id -1, score 0."""
    keys = np.asarray(keys, dtype=np.int64)
    valid = keys != np.iinfo(np.int64).min
    ids = np.where(valid, ((1 << 31) - 1) - (keys & 0xFFFFFFFF), -1)
    scores = np.where(valid, keys >> 32, 0)
    return ids.astype(np.int64), scores.astype(np.int64)
