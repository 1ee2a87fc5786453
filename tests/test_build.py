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

INCDIRS = (CSRC, os.path.join(REPO, "include"))
INCLUDE_RE = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)
# translation units the Makefile compiles, and the object each one makes
HOST_TUS = ("main.cpp", "swsolver.cpp", "sw_tests.cpp")


def _obj(src):
    stem = src.rsplit(".", 1)[0]
    return stem + (".host.o" if src in HOST_TUS else ".o")


def _resolve(name, from_dir):
    for d in (from_dir,) + INCDIRS:
        path = os.path.normpath(os.path.join(d, name))
        if os.path.exists(path):
            return path
    return None


def _closure(path, seen=None):
    """Every in-tree header PATH includes, transitively (the preprocessor's
    search order for quoted includes: the including file's directory, then
    the -I directories)."""
    seen = set() if seen is None else seen
    for name in INCLUDE_RE.findall(open(path).read()):
        dep = _resolve(name, os.path.dirname(path))
        if dep and dep not in seen:
            seen.add(dep)
            _closure(dep, seen)
    return seen


def includers():
    """header path -> the objects whose translation units include it,
    derived from the sources (no hand-kept table: round 4's sw_int32.h was
    missing from one)."""
    table = {}
    for src in sorted(os.listdir(CSRC)):
        if src.endswith((".hip", ".cpp")):
            for hdr in _closure(os.path.join(CSRC, src)):
                table.setdefault(hdr, set()).add(_obj(src))
    return table


def would_rebuild(header):
    out = subprocess.run(["make", "-n", "-C", CSRC, "ARCH=gfx950", "-W", header],
                         check=True, capture_output=True, text=True).stdout
    return set(re.findall(r"-o \S*/(\w+(?:\.host)?\.o) ", out))


def test_every_header_has_includers():
    # the derivation sees the kernel headers (sw_int32.h is included by two
    # kernel sources, sw_intra_x2.h by two, sw_kernels.h transitively by all)
    table = {os.path.basename(h): objs for h, objs in includers().items()}
    assert {"sw_kernels.o", "sw_inter_x2.o"} <= table["sw_int32.h"]
    assert {"sw_intra_x2.o", "sw_inter_x2.o"} <= table["sw_intra_x2.h"]
    assert {"sw_capi.o", "sw_group.o", "sw_topk.o", "sw_align.o"} <= table["sw_kernels.h"]
    assert {"main.host.o", "swsolver.host.o", "sw_tests.host.o"} <= table["FASTAParsers.h"]
    every = {os.path.basename(p) for p in os.listdir(CSRC) if p.endswith(".h")}
    every |= {p for p in os.listdir(INCDIRS[1]) if p.endswith(".h")}
    assert every <= set(table), every - set(table)


@pytest.mark.skipif(shutil.which("make") is None, reason="no make")
@pytest.mark.parametrize("header", sorted(os.path.relpath(h, REPO) for h in includers()))
def test_header_change_rebuilds_its_objects(header):
    """`make -n -W header` rebuilds every object whose source includes the
    header, directly or through another header (the Makefile's generated
    -MMD dependencies; an object built without its .d is rebuilt)."""
    objs = includers()[os.path.join(REPO, header)]
    missing = objs - would_rebuild(os.path.join(REPO, header))
    assert not missing, (header, missing)


PKG_NAME = "ece1782-smith-waterman-cuda_amd"
LOAD = ("import sys; sys.path.insert(0, sys.argv[1]); import _swpkg; sw = _swpkg.load(); "
        "print('build id', sw.capi.build_id())")


def _load_in(root):
    return subprocess.run([__import__("sys").executable, "-c", LOAD, str(root)], capture_output=True, text=True,
                          timeout=300)


@pytest.mark.skipif(shutil.which("make") is None, reason="no make")
@pytest.mark.parametrize("edited", ["csrc/main.cpp", "csrc/sw_int32.h"])
def test_stale_library_is_refused_until_rebuilt(tmp_path, edited):
    """The library carries the id of the sources it was built from
    (sw_build_id, csrc/build_id.py); the Python binding refuses a library
    whose id is not the tree's, and make rebuilds it when any source changes
    (the id stamp, not mtimes).  Run on a copy of the tree (objects and their
    generated .d files included, so only the changed pieces recompile): an
    edit to a kernel header must recompile exactly the objects that include
    it, in the copy (the .d files name $(OBJ)/$(ROOT), not this tree)."""
    root = tmp_path / "repo"
    shutil.copytree(os.path.join(REPO, PKG_NAME), root / PKG_NAME, symlinks=True,
                    ignore=shutil.ignore_patterns("__pycache__"))
    shutil.copytree(os.path.join(REPO, "include"), root / "include")
    shutil.copy(os.path.join(REPO, "_swpkg.py"), root)
    ok = _load_in(root)
    assert ok.returncode == 0, ok.stderr
    built = ok.stdout.split()[-1]
    obj_dir = root / PKG_NAME / "lib" / "obj"
    before = {p.name: p.stat().st_mtime_ns for p in obj_dir.glob("*.o")}
    src = root / PKG_NAME / edited
    src.write_text(src.read_text() + "// a change to one source\n")
    stale = _load_in(root)
    assert stale.returncode != 0 and "stale HIP library" in stale.stderr, stale.stderr
    subprocess.run(["make", "-s", "-j", "8", "-C", str(root / PKG_NAME / "csrc"), "ARCH=gfx950"], check=True,
                   capture_output=True, timeout=900)
    fresh = _load_in(root)
    assert fresh.returncode == 0, fresh.stderr
    assert fresh.stdout.split()[-1] != built
    rebuilt = {p.name for p in obj_dir.glob("*.o") if p.stat().st_mtime_ns != before.get(p.name)}
    expect = includers()[os.path.join(CSRC, os.path.basename(edited))] if edited.endswith(".h") else {"main.host.o"}
    # sw_capi.o also recompiles: it carries the new source id
    assert rebuilt == expect | {"sw_capi.o"}, rebuilt
