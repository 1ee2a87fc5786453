"""Python mirror of the reference's solver interface (SWSolver.h / SWSolver_char.h).

    smith_waterman_cuda(query, db, result)        SWSolver.h:9, SWSolver.cu:266-404
    smith_waterman_cuda_char(query, db) -> list   SWSolver_char.h:9, SWSolver_char.cu:193-280

Same argument meaning and result semantics as the reference:
* the query is padded with '/' to a multiple of 8 before scoring
  (SWSolver.cu:267-269) and every sequence of the database is used as parsed
  (already '/'-padded, FASTAParsers.h:94-96); '/' scores as '*', i.e. 0
  under the reference BLOSUM50 (SWSolver.cu:80,119), so padding never moves a
  score;
* `result` receives (id, score) pairs APPENDED (SWSolver.cu:387) in descending
  padded-length order, file order within a length (SWSolver.cu:309,384-390).
The char variant (which does not compile in the reference)
returns the same scores as a fresh list in file order; in compat mode
(SW_CHAR_COMPAT=1) it scores as the char path's own table
would: '*' (and what its encoder maps to '*': the parser's '/' padding, U, O,
lowercase) -5 against a letter, +1 against '*', the query unpadded.

Differences, on purpose: scores are exact int32 (the reference stores int16
and would overflow); there is no 1024-residue query cap
(SWSolver.cu:85, F6); HIP errors raise instead of being ignored
(SWSolver.cu:276).
"""
import os
import numpy as np

from . import capi
from .fasta import TILE_SIZE

_HANDLE = None


def default_handle():
    global _HANDLE
    if _HANDLE is None:
        _HANDLE = capi.Handle(0, env_opts=False)
    return _HANDLE


def _padded_query(query):
    q = query.get_buffer()
    while len(q) % TILE_SIZE != 0:  # SWSolver.cu:268-269
        q = q + "/"
    return q


def _scores_by_record(query, db, handle=None, pad=True, **scoring):
    h = handle or default_handle()
    residues, offsets, ids = db.flat(capi.encode)
    # Record ids may repeat only for the degenerate -1 case; key by position.
    gdb = capi.Database(h, residues, offsets)
    q = _padded_query(query) if pad else query.get_buffer()
    scores = gdb.scan(capi.encode(q), **scoring)
    gdb.close()
    return ids, scores


def smith_waterman_cuda(query, db, result, handle=None):
    """Append (id, best local score) for every subject of `db` to `result`."""
    ids, scores = _scores_by_record(query, db, handle)
    pos = {}
    for k, (i, _) in enumerate(db.records()):
        pos.setdefault(i, []).append(k)
    taken = {}
    for length in sorted(db.parsedDB, reverse=True):  # map reverse iteration, SWSolver.cu:309
        for subj in db.parsedDB[length]:
            j = taken.get(subj.id, 0)
            k = pos[subj.id][j]
            taken[subj.id] = j + 1
            result.append((subj.id, int(scores[k])))
    return None


def smith_waterman_cuda_char(query, db, handle=None, compat=None):
    """Same scores, returned as a new list in file order.  compat (default:
    env SW_CHAR_COMPAT == "1", as the C++ shim): score with the _char path's
    own table instead — BLOSUM50 with '*' = -5 (SWSolver_char.cu:22-49 read
    through its lookup :106-179) — and the query unpadded."""
    if compat is None:
        compat = os.environ.get("SW_CHAR_COMPAT") == "1"
    if compat:
        ids, scores = _scores_by_record(query, db, handle, pad=False,
                                        matrix=capi.builtin_matrix(capi.MATRIX_BLOSUM50_CHAR), gap_open=2)
    else:
        ids, scores = _scores_by_record(query, db, handle)
    return [(int(i), int(s)) for i, s in zip(ids, scores)]
