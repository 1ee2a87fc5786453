"""GPU: the drop-in C++ path — bin/main and the swissprot_tests harness —
end to end through the HIP library, against the golden scores."""
import os
import subprocess

import pytest

from conftest import GOLDEN, REPO, read_golden

pytestmark = pytest.mark.gpu
LIB = os.path.join(REPO, "ece1782-smith-waterman-cuda_amd", "lib")


@pytest.mark.parametrize("qname", ["P01008", "P02232"])
def test_main_cli_output(qname):
    out = subprocess.run([os.path.join(LIB, "main"), "--query", GOLDEN + "/queries/%s.fasta" % qname,
                          "--db", GOLDEN + "/subset111.fasta"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.split("\n")
    assert lines[0].startswith("Input buffer:")
    pairs = [tuple(map(int, ln.split(":"))) for ln in lines if ln and ln[0].isdigit() and ":" in ln]
    golden = read_golden(qname + ".subset111.scores")
    assert len(pairs) == 111
    assert all(golden[i] == s for i, s in pairs)
    assert "METRICS:" in out.stdout and "GCUPS." in out.stdout
    assert "Num subjects: 111" in out.stdout


def test_swissprot_harness():
    out = subprocess.run([os.path.join(LIB, "sw_tests"), "--suite", "all"], capture_output=True, text=True,
                         cwd=REPO, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 failure(s)" in out.stdout
    assert out.stdout.count("GCUPS") == 17
