"""FASTA input contract, mirroring the reference's src/FASTAParsers.h.

Same classes, fields and behaviour as the header (FASTAParsers.h:16-138),
including its edge cases, so code written against the reference reads the
same here:

* FASTAQuery(path, isQuery): skips the first line and concatenates every
  remaining line verbatim (FASTAParsers.h:38-51).
* FASTADatabase(path): a '>' line starts a record; record ids are 0-based in
  file order (FASTAParsers.h:82,98,112); each sequence is padded with '/' to a
  multiple of TILE_SIZE = 8 (FASTAParsers.h:12,94-96,120-122) and bucketed by
  padded length in `parsedDB` (FASTAParsers.h:68,101,129); `subjectLengthSum`
  sums PADDED lengths (FASTAParsers.h:103,131).  Lines before the first '>'
  are dropped; a file with no '>' becomes ONE subject with id -1; an empty
  file yields one empty subject with id -1 (FASTAParsers.h:78-134).

`flat()` gives the encoded, concatenated form the C ABI takes (sw_db_create).
"""
import numpy as np

TILE_SIZE = 8


def round_up(num, multiple):
    """FASTAParsers.h:21-31."""
    if multiple == 0:
        return num
    rem = num % multiple
    return num if rem == 0 else num + multiple - rem


class SubjectSequence:
    """FASTAParsers.h:16-19."""
    __slots__ = ("id", "sequence")

    def __init__(self, id_, sequence):
        self.id = id_
        self.sequence = sequence

    def __repr__(self):
        return "SubjectSequence(id=%d, len=%d)" % (self.id, len(self.sequence))


def _lines(path):
    # getline semantics: split on '\n' only; a trailing newline does not
    # produce an extra empty line.
    with open(path, "rb") as f:
        data = f.read().decode("latin-1")
    if not data:
        return []
    parts = data.split("\n")
    if parts[-1] == "":
        parts.pop()
    return parts


class FASTAQuery:
    """FASTAParsers.h:33-63."""

    def __init__(self, filepath, isQuery=True):
        self.isQuery = isQuery
        lines = _lines(filepath)
        self.buffer = "".join(lines[1:])

    def print_buffer(self):
        print(self.buffer)

    def get_buffer(self):
        return self.buffer


class FASTADatabase:
    """FASTAParsers.h:65-138."""

    def __init__(self, filepath):
        self.parsedDB = {}
        self.largestSubjectLength = 0
        self.numSubjects = 0
        self.subjectLengthSum = 0
        self._records = []  # (id, padded sequence) in file order
        _id = -1
        is_first = True
        seq = []
        for line in _lines(filepath):
            if line[:1] == ">":
                if not is_first:
                    self._add(_id, "".join(seq))
                is_first = False
                seq = []
                _id += 1
            else:
                seq.append(line)
        self._add(_id, "".join(seq))  # FASTAParsers.h:117-134: always adds the last record

    def _add(self, id_, s):
        s = s + "/" * (round_up(len(s), TILE_SIZE) - len(s))
        self.parsedDB.setdefault(len(s), []).append(SubjectSequence(id_, s))
        self._records.append((id_, s))
        self.subjectLengthSum += len(s)
        self.largestSubjectLength = max(self.largestSubjectLength, len(s))
        self.numSubjects += 1

    def records(self):
        """(id, padded sequence) in file order."""
        return list(self._records)

    def flat(self, encode):
        """Encoded residues, int64 offsets (n+1) and the record ids, file order."""
        seqs = [s for _, s in self._records]
        joined = "".join(seqs)
        residues = encode(joined) if joined else np.zeros(0, dtype=np.uint8)
        offsets = np.zeros(len(seqs) + 1, dtype=np.int64)
        offsets[1:] = np.cumsum([len(s) for s in seqs])
        ids = np.array([i for i, _ in self._records], dtype=np.int64)
        return residues, offsets, ids
