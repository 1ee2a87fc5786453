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
