"""CPU: the FASTA input contract (reference FASTAParsers.h) — the Python
mirror and the C++ drop-in header agree with each other and with the
reference header's documented behaviour, including its edge cases."""
import os
import subprocess

import pytest

from conftest import GOLDEN, REPO

CASES = {
    "normal": ">a\nACDE\nFG\n>b\n\n>c\nWWWWWWWWW\n",
    "no_header": "ACGT\nACGT\n",
    "empty": "",
    "preamble": "junk\n>x\nMKV\n",
    "crlf": ">x\r\nMKV\r\n>y\r\nAA\r\n",
    "no_trailing_newline": ">x\nMKVLA",
    "blank_lines": ">x\nMK\n\nVL\n>y\n",
}

PRINTER = r"""
#include "FASTAParsers.h"
int main(int argc, char** argv) {
    FASTADatabase db(argv[1]);
    FASTAQuery q(argv[1], true);
    cout << db.numSubjects << " " << db.subjectLengthSum << " " << db.largestSubjectLength << "\n";
    for (map<int, vector<subject_sequence> >::iterator it = db.parsedDB.begin(); it != db.parsedDB.end(); ++it)
        for (size_t i = 0; i < it->second.size(); ++i)
            cout << it->first << " " << it->second[i].id << " [" << it->second[i].sequence << "]\n";
    cout << "Q[" << q.get_buffer() << "]\n";
    return 0;
}
"""


def python_dump(sw, path):
    db = sw.FASTADatabase(path)
    q = sw.FASTAQuery(path, True)
    lines = ["%d %d %d" % (db.numSubjects, db.subjectLengthSum, db.largestSubjectLength)]
    for L in sorted(db.parsedDB):
        for s in db.parsedDB[L]:
            lines.append("%d %d [%s]" % (L, s.id, s.sequence))
    lines.append("Q[%s]" % q.get_buffer())
    return "\n".join(lines) + "\n"


@pytest.fixture(scope="module")
def printer(tmp_path_factory):
    d = tmp_path_factory.mktemp("fasta")
    src = d / "p.cpp"
    src.write_text(PRINTER)
    exe = d / "p"
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(REPO, "include"), "-o", str(exe), str(src)],
                   check=True)
    return str(exe)


@pytest.mark.parametrize("name", sorted(CASES))
def test_cpp_header_equals_python_mirror(sw, printer, tmp_path, name):
    p = tmp_path / (name + ".fa")
    p.write_bytes(CASES[name].encode())
    cpp = subprocess.run([printer, str(p)], capture_output=True, check=True).stdout.decode("latin-1")
    assert cpp == python_dump(sw, str(p))


def test_documented_behaviour(sw, tmp_path):
    p = tmp_path / "n.fa"
    p.write_text(CASES["normal"])
    db = sw.FASTADatabase(str(p))
    assert db.numSubjects == 3
    assert [(s.id, s.sequence) for s in db.parsedDB[8]] == [(0, "ACDEFG//")]
    assert db.parsedDB[0][0].id == 1                          # empty record kept
    assert db.parsedDB[16][0].sequence == "W" * 9 + "/" * 7
    assert db.subjectLengthSum == 24                          # padded lengths
    p.write_text(CASES["no_header"])
    db = sw.FASTADatabase(str(p))
    assert db.numSubjects == 1 and db.parsedDB[8][0].id == -1
    p.write_text("")
    db = sw.FASTADatabase(str(p))
    assert db.numSubjects == 1 and db.parsedDB[0][0].id == -1 and db.parsedDB[0][0].sequence == ""


def test_subset_fixture(sw):
    db = sw.FASTADatabase(GOLDEN + "/subset111.fasta")
    assert db.numSubjects == 111
    assert sorted(i for i, _ in db.records()) == list(range(111))
    q = sw.FASTAQuery(GOLDEN + "/queries/P02232.fasta", True)
    assert len(q.get_buffer()) == 144


def test_flat_encoding(sw):
    db = sw.FASTADatabase(GOLDEN + "/subset111.fasta")
    res, offs, ids = db.flat(sw.encode)
    assert len(offs) == 112 and offs[-1] == db.subjectLengthSum == len(res)
    assert ids.tolist() == list(range(111))
