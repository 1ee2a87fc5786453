"""MI355X-native Smith-Waterman database search (drop-in for the reference's
smith_waterman_cuda scan path).

Product path: lib/libswamd.so (HIP kernels for gfx950 + host driver) behind
the C ABI in include/sw_amd.h, with C++ shims (include/SWSolver.h) and this
Python face.  There is no CPU fallback: if the library is missing, calls raise.

Load with `import sw_amd` after `_swpkg.load()` (the directory name carries
hyphens, so it is registered under the module name `sw_amd`).
"""
from . import capi, dist, fasta, solver, synth  # noqa: F401
from .capi import Database, Group, Handle, SWError, builtin_matrix, encode, topk  # noqa: F401
from .fasta import FASTADatabase, FASTAQuery, SubjectSequence  # noqa: F401
from .solver import smith_waterman_cuda, smith_waterman_cuda_char  # noqa: F401

MATRIX_BLOSUM50_REF = capi.MATRIX_BLOSUM50_REF
MATRIX_BLOSUM62 = capi.MATRIX_BLOSUM62
MATRIX_IDENTITY3 = capi.MATRIX_IDENTITY3
MATRIX_BLOSUM50_CHAR = capi.MATRIX_BLOSUM50_CHAR
