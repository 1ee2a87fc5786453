"""The in-tree build (csrc/Makefile, driven by __graft_entry__.build()):
every object that compiles a header's code is rebuilt when that header
changes.  Round 3 lost GPU time to a stale library: sw_intra_x2.h (the intra
kernel body, also compiled into the merged launch in sw_inter_x2.hip) was
missing from the dependencies, so header-only edits did not rebuild.
`make -n -W FILE` lists what a newer FILE would rebuild without touching
anything."""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "ece1782-smith-waterman-cuda_amd", "csrc")

# header -> the objects whose translation units include it
INCLUDERS = {
    "sw_intra_x2.h": {"sw_intra_x2.o", "sw_inter_x2.o"},
    "sw_kernels.h": {"sw_kernels.o", "sw_inter_x2.o", "sw_intra_x2.o", "sw_align.o", "sw_synth.o",
                     "sw_profile.o", "sw_topk.o", "sw_capi.o", "sw_group.o"},
}


def would_rebuild(header):
    out = subprocess.run(["make", "-n", "-C", CSRC, "ARCH=gfx950", "-W", os.path.join(CSRC, header)],
                         check=True, capture_output=True, text=True).stdout
    return set(re.findall(r"-o \S*/(sw_\w+\.o) ", out))


@pytest.mark.skipif(shutil.which("make") is None, reason="no make")
@pytest.mark.parametrize("header", sorted(INCLUDERS))
def test_header_change_rebuilds_its_objects(header):
    assert INCLUDERS[header] <= would_rebuild(header)


def test_includers_table_matches_the_sources():
    # every csrc translation unit that includes a header is listed for it
    for header, objs in INCLUDERS.items():
        for src in os.listdir(CSRC):
            if not src.endswith((".hip", ".cpp")) or src in ("main.cpp", "swsolver.cpp", "sw_tests.cpp"):
                continue
            text = open(os.path.join(CSRC, src)).read()
            direct = '#include "%s"' % header in text
            via_ix2 = header == "sw_kernels.h" and '#include "sw_intra_x2.h"' in text
            if direct or via_ix2:
                assert src.rsplit(".", 1)[0] + ".o" in objs, (header, src)


PKG_NAME = "ece1782-smith-waterman-cuda_amd"
LOAD = ("import sys; sys.path.insert(0, sys.argv[1]); import _swpkg; sw = _swpkg.load(); "
        "print('build id', sw.capi.build_id())")


def _load_in(root):
    return subprocess.run([__import__("sys").executable, "-c", LOAD, str(root)], capture_output=True, text=True,
                          timeout=300)


@pytest.mark.skipif(shutil.which("make") is None, reason="no make")
def test_stale_library_is_refused_until_rebuilt(tmp_path):
    """The library carries the id of the sources it was built from
    (sw_build_id, csrc/build_id.py); the Python binding refuses a library
    whose id is not the tree's, and make rebuilds it when any source changes
    (the id stamp, not mtimes).  Run on a copy of the tree (objects included,
    so only the changed pieces recompile)."""
    root = tmp_path / "repo"
    shutil.copytree(os.path.join(REPO, PKG_NAME), root / PKG_NAME, symlinks=True,
                    ignore=shutil.ignore_patterns("__pycache__"))
    shutil.copytree(os.path.join(REPO, "include"), root / "include")
    shutil.copy(os.path.join(REPO, "_swpkg.py"), root)
    ok = _load_in(root)
    assert ok.returncode == 0, ok.stderr
    built = ok.stdout.split()[-1]
    main_cpp = root / PKG_NAME / "csrc" / "main.cpp"
    main_cpp.write_text(main_cpp.read_text() + "// a change to one source\n")
    stale = _load_in(root)
    assert stale.returncode != 0 and "stale HIP library" in stale.stderr, stale.stderr
    subprocess.run(["make", "-s", "-j", "8", "-C", str(root / PKG_NAME / "csrc"), "ARCH=gfx950"], check=True,
                   capture_output=True, timeout=600)
    fresh = _load_in(root)
    assert fresh.returncode == 0, fresh.stderr
    assert fresh.stdout.split()[-1] != built
