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


def _pairs(stdout):
    return [tuple(map(int, ln.split(":"))) for ln in stdout.split("\n") if ln and ln[0].isdigit() and ":" in ln]


def test_binary_db_cli_same_output(tmp_path):
    """--make-db writes the FASTA as a .swdb file; scanning it prints the
    same id:score lines in the same order, and the same METRICS sizes."""
    swdb = str(tmp_path / "subset111.swdb")
    mk = subprocess.run([os.path.join(LIB, "main"), "--make-db", swdb, "--db", GOLDEN + "/subset111.fasta"],
                        capture_output=True, text=True, timeout=300)
    assert mk.returncode == 0, mk.stderr
    runs = []
    for db in (GOLDEN + "/subset111.fasta", swdb):
        out = subprocess.run([os.path.join(LIB, "main"), "--query", GOLDEN + "/queries/P01008.fasta", "--db", db],
                             capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stderr
        runs.append(out.stdout)
    assert _pairs(runs[0]) == _pairs(runs[1])
    for key in ("Num subjects:", "Sum of DB length:", "Query length:"):
        assert [ln for ln in runs[0].split("\n") if ln.startswith(key)] == \
               [ln for ln in runs[1].split("\n") if ln.startswith(key)]


def test_binary_db_rejects_corruption(tmp_path):
    swdb = str(tmp_path / "x.swdb")
    subprocess.run([os.path.join(LIB, "main"), "--make-db", swdb, "--db", GOLDEN + "/subset111.fasta"],
                   capture_output=True, text=True, timeout=300, check=True)
    data = bytearray(open(swdb, "rb").read())
    data[-10] ^= 0x01  # flip one residue bit
    bad = str(tmp_path / "bad.swdb")
    open(bad, "wb").write(bytes(data))
    out = subprocess.run([os.path.join(LIB, "main"), "--query", GOLDEN + "/queries/P01008.fasta", "--db", bad],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode != 0 and "checksum" in out.stderr
