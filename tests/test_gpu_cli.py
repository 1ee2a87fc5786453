"""GPU: the drop-in C++ path — bin/main and the swissprot_tests harness —
end to end through the HIP library, against the golden scores."""
import os
import subprocess

import numpy as np
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


def _run(args, timeout=300, env=None):
    out = subprocess.run([os.path.join(LIB, "main")] + args, capture_output=True, text=True, timeout=timeout, env=env)
    assert out.returncode == 0, out.stderr
    return out.stdout


def _oracle_scores(oracle, qname, path, mat, go, ge, pad):
    from conftest import read_query
    q = read_query(qname)
    if pad:
        q += "/" * (-len(q) % 8)  # SWSolver.cu:267-269 (the reference's scoring only)
    recs = oracle.read_fasta_records(path)
    res = np.concatenate([oracle.encode(s) for _, s in recs]) if recs else np.zeros(0, np.uint8)
    offs = np.zeros(len(recs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(s) for _, s in recs])
    return oracle.scan(oracle.encode(q), res, offs, mat=mat, gap_open=go, gap_extend=ge, nthreads=16)


def _topk(scores, k):
    order = np.lexsort((np.arange(len(scores)), -np.asarray(scores, dtype=np.int64)))[:k]
    return [(int(i), int(scores[i])) for i in order]


def _write_ncbi(path, mat, letters="ARNDCQEGHILKMFPSTWYVBJZX*"):
    codes = ["ARNDCQEGHILKMFPSTWYVBJZX*".index(c) for c in letters]
    with open(path, "w") as f:
        f.write("# a BLOSUM62 in NCBI's layout\n   " + "  ".join(letters) + "\n")
        for a in codes:
            f.write("ARNDCQEGHILKMFPSTWYVBJZX*"[a] + " " + " ".join("%2d" % mat[a][b] for b in codes) + "\n")


@pytest.mark.parametrize("qname", ["P01008", "P02232"])
def test_main_scoring_flags(sw, oracle, tmp_path, qname):
    """main --matrix blosum62 --gap-open 12 --gap-extend 1 (the headline
    scoring, BLAST 11/1) on the 111-record subset equals the oracle; a matrix
    file in NCBI's layout and a 25x25 code-order file give the same scores
    as the built-in tables they hold."""
    db = GOLDEN + "/subset111.fasta"
    qf = GOLDEN + "/queries/%s.fasta" % qname
    m62 = sw.capi.builtin_matrix(1)
    want = _oracle_scores(oracle, qname, db, m62, 12, 1, pad=False)
    got = dict(_pairs(_run(["--query", qf, "--db", db, "--matrix", "blosum62", "--gap-open", "12",
                            "--gap-extend", "1"])))
    assert len(got) == 111 and [got[i] for i in range(111)] == list(want)
    ncbi = str(tmp_path / "b62.txt")
    _write_ncbi(ncbi, m62)
    got2 = dict(_pairs(_run(["--query", qf, "--db", db, "--matrix=" + ncbi, "--gap-open=12", "--gap-extend=1"])))
    assert got2 == got
    plain = str(tmp_path / "id3.txt")
    m3 = sw.capi.builtin_matrix(2)
    with open(plain, "w") as f:
        f.write("\n".join(" ".join(str(int(v)) for v in row) for row in m3) + "\n")
    want3 = _oracle_scores(oracle, qname, db, m3, 3, 3, pad=False)
    got3 = dict(_pairs(_run(["--query", qf, "--db", db, "--matrix", plain, "--gap-open", "3"])))
    assert [got3[i] for i in range(111)] == list(want3)


def test_main_ncbi_matrix_without_j_scores_j_as_x(sw, tmp_path):
    """NCBI's own BLOSUM62 file has no J: J then scores as X (documented in
    sw_solver_ext.h); the subset holds no J, so the scores equal the
    built-in BLOSUM62's."""
    db = GOLDEN + "/subset111.fasta"
    qf = GOLDEN + "/queries/P02232.fasta"
    path = str(tmp_path / "ncbi62.txt")
    _write_ncbi(path, sw.capi.builtin_matrix(1), letters="ARNDCQEGHILKMFPSTWYVBZX*")
    a = _pairs(_run(["--query", qf, "--db", db, "--matrix", path, "--gap-open", "12", "--gap-extend", "1"]))
    b = _pairs(_run(["--query", qf, "--db", db, "--matrix", "blosum62", "--gap-open", "12", "--gap-extend", "1"]))
    assert a == b


@pytest.mark.parametrize("scoring", [[], ["--matrix", "blosum62", "--gap-open", "12", "--gap-extend", "1"]])
def test_main_topk(sw, oracle, tmp_path, scoring):
    """--topk K prints the oracle's top-K (score descending, record id
    ascending) in rank order, from the FASTA and from a .swdb file; K larger
    than the database prints every subject ranked; the default output (no
    flags) still equals the golden file (test_main_cli_output)."""
    db = GOLDEN + "/subset111.fasta"
    qf = GOLDEN + "/queries/P01008.fasta"
    custom = bool(scoring)
    mat = sw.capi.builtin_matrix(1 if custom else 0)
    want = _oracle_scores(oracle, "P01008", db, mat, 12 if custom else 2, 1 if custom else 2, pad=not custom)
    swdb = str(tmp_path / "s.swdb")
    subprocess.run([os.path.join(LIB, "main"), "--make-db", swdb, "--db", db], check=True, capture_output=True,
                   timeout=300)
    for src in (db, swdb):
        for k in (1, 10, 100, 500, 5000):
            got = _pairs(_run(["--query", qf, "--db", src, "--topk", str(k)] + scoring))
            assert got == _topk(want, k), (src, k)


def test_main_chosen_scoring_scans_sequences_as_written(sw, oracle, tmp_path):
    """Under a chosen scoring the query and the subjects are scanned as
    written: the reference's '/' padding (SWSolver.cu:267-269,
    FASTAParsers.h) encodes as '*', which BLOSUM62 scores +1 against '*', so
    a query ending in U ('*') would gain a point on every padded subject.
    FASTA and .swdb paths both equal the oracle on the raw sequences."""
    from conftest import read_query
    base = read_query("P02232")  # 144 aa
    qtext = base + "U"
    qf = str(tmp_path / "q.fasta")
    with open(qf, "w") as f:
        f.write(">query ending in U\n" + qtext + "\n")
    subjects = [base[:-1], base[:100] + "U", base[20:90], "MKV"]
    dbf = str(tmp_path / "db.fasta")
    with open(dbf, "w") as f:
        for k, t in enumerate(subjects):
            f.write(">s%d\n%s\n" % (k, t))
    m = sw.capi.builtin_matrix(1)
    res = np.concatenate([oracle.encode(t) for t in subjects])
    offs = np.zeros(len(subjects) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(t) for t in subjects])
    want = oracle.scan(oracle.encode(qtext), res, offs, mat=m, gap_open=12, gap_extend=1)
    flags = ["--matrix", "blosum62", "--gap-open", "12", "--gap-extend", "1"]
    swdb = str(tmp_path / "db.swdb")
    subprocess.run([os.path.join(LIB, "main"), "--make-db", swdb, "--db", dbf], check=True, capture_output=True,
                   timeout=300)
    for src in (dbf, swdb):
        got = dict(_pairs(_run(["--query", qf, "--db", src] + flags)))
        assert [got[i] for i in range(len(subjects))] == list(want), src
