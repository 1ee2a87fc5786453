"""CPU: the drop-in CLI and harness build and handle their arguments like
the reference's (usage + exit 1 without --query/--db, main.cpp:33-41)."""
import os
import subprocess

import pytest

from conftest import REPO

LIB = os.path.join(REPO, "ece1782-smith-waterman-cuda_amd", "lib")


@pytest.mark.parametrize("args", [[], ["--help"], ["--query", "x.fasta"], ["--db", "y"]])
def test_main_usage(args):
    out = subprocess.run([os.path.join(LIB, "main")] + args, capture_output=True, text=True)
    assert out.returncode == 1
    assert "--query" in out.stdout and "--db" in out.stdout


def test_main_unknown_option():
    out = subprocess.run([os.path.join(LIB, "main"), "--frobnicate", "1"], capture_output=True, text=True)
    assert out.returncode == 1


def test_binaries_link_the_hip_library():
    for exe in ("main", "sw_tests"):
        out = subprocess.run(["ldd", os.path.join(LIB, exe)], capture_output=True, text=True).stdout
        assert "libswamd.so" in out


@pytest.mark.parametrize("flags, msg", [
    (["--matrix", "/nonexistent/matrix.txt"], "--matrix"),
    (["--matrix", "blosum62", "--gap-open", "0"], "--gap-open"),
    (["--gap-open", "12", "--gap-extend", "x"], "--gap-extend"),
    (["--topk", "0"], "--topk"),
])
def test_main_bad_scoring_flags(flags, msg):
    """Scoring / top-K flags are checked before any file is read or any GPU
    is touched: a bad value exits 1 with a message naming the flag."""
    out = subprocess.run([os.path.join(LIB, "main"), "--query", "q.fasta", "--db", "d.fasta"] + flags,
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 1 and msg in out.stderr, out.stderr


def test_main_matrix_file_errors(tmp_path):
    bad = tmp_path / "m.txt"
    for text, msg in (("A R\nA 1 2\nR 2 1\n", "no row for"), ("A R\nA 1 2\n", "row or a column"),
                      ("1 2 3\n", "25 rows"), ("A R\nA 1 x\nR 1 1\n", "bad entry"),
                      ("A Q9\nA 1 2\n", "unknown residue letter")):
        bad.write_text(text)
        out = subprocess.run([os.path.join(LIB, "main"), "--query", "q.fasta", "--db", "d.fasta", "--matrix",
                              str(bad)], capture_output=True, text=True, timeout=60)
        assert out.returncode == 1 and msg in out.stderr, (text, out.stderr)
