#!/usr/bin/env python3
"""The source id compiled into libswamd.so (sw_build_id) and checked by
capi.py when the library is loaded: the first 16 hex digits of a SHA-256
over every source the library and tools are built from — csrc/*.{hip,cpp,h},
csrc/Makefile, this script and include/*.h — in sorted order, each as
"<dir>/<name>\\0<bytes>".  A library whose id differs from the tree's
sources is stale (built from other sources) and is refused.

Usage: build_id.py [REPO_ROOT]   prints the id (the Makefile's stamp)."""
import hashlib
import os
import sys

_PKG = "ece1782-smith-waterman-cuda_amd"


def source_files(root):
    csrc = os.path.join(root, _PKG, "csrc")
    inc = os.path.join(root, "include")
    out = []
    for name in sorted(os.listdir(csrc)):
        if name.endswith((".hip", ".cpp", ".h")) or name in ("Makefile", "build_id.py"):
            out.append(("csrc/" + name, os.path.join(csrc, name)))
    for name in sorted(os.listdir(inc)):
        if name.endswith(".h"):
            out.append(("include/" + name, os.path.join(inc, name)))
    return out


def source_id(root):
    h = hashlib.sha256()
    for rel, path in source_files(root):
        with open(path, "rb") as f:
            h.update(rel.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    print(source_id(sys.argv[1] if len(sys.argv) > 1 else os.path.dirname(os.path.dirname(here))))
