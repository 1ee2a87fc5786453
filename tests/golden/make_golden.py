#!/usr/bin/env python3
"""Regenerate the committed golden fixtures from the reference tree.

Runs ONLY in the build container (it reads /root/reference, which does not
exist on the GPU box).  Everything it writes is data: inputs and expected
outputs.  No reference source text is copied.

  subset111.fasta              data/dbs/uniprot_subset.dat (UniProt flat file,
                               the first 111 SwissProt entries) as FASTA, one
                               record per entry, in file order.  Record k of
                               this file is record k of uniprot_sprot.fasta.
  P01008.subset111.scores      lines 0..110 of test/reference/P01008.txt
  P02232.subset111.scores      lines 0..110 of test/reference/P02232.txt
  P01008.full.txt.gz           the whole golden files (559,228 scores each),
  P02232.full.txt.gz           for the SwissProt-wide test when a user
                               supplies uniprot_sprot.fasta (SW_SWISSPROT env)
  queries/*.fasta              data/queries/*.fasta, byte for byte
  cpu_pairs.json               outputs of the reference's src/cpu.cpp
                               (compiled untouched into oracle/_ref/cpu_ref by
                               `make -C oracle ref`) on seeded pairs: the two
                               alignment rows it prints and the maximum of the
                               matrix it prints.

Usage:  make -C oracle ref && python tests/golden/make_golden.py
"""
import gzip
import json
import os
import random
import shutil
import subprocess
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def uniprot_dat_to_fasta(path):
    """Parse UniProt flat-file records: ID/AC lines, SQ line, sequence lines
    up to '//' (or EOF for the last, unterminated record)."""
    recs = []
    ident, acc, seq, in_sq = None, None, [], False
    with open(path) as f:
        for line in f:
            if line.startswith("ID   "):
                ident = line.split()[1]
            elif line.startswith("AC   ") and acc is None:
                acc = line.split()[1].rstrip(";")
            elif line.startswith("SQ   "):
                in_sq, seq = True, []
            elif line.startswith("//"):
                recs.append((acc, ident, "".join(seq)))
                ident, acc, seq, in_sq = None, None, [], False
            elif in_sq:
                seq.append("".join(line.split()))
    if in_sq:
        recs.append((acc, ident, "".join(seq)))
    return recs


def write_fasta(recs, path, width=60):
    with open(path, "w") as f:
        for acc, ident, seq in recs:
            f.write(">sp|%s|%s\n" % (acc, ident))
            for k in range(0, len(seq), width):
                f.write(seq[k:k + width] + "\n")


def cpu_ref_pair(binary, a, b):
    out = subprocess.run([binary, a, b], capture_output=True, text=True, check=True).stdout
    lines = out.split("\n")
    aln_a, aln_b = lines[0], lines[1]
    best = 0
    for ln in lines[3:]:  # line 2 is the column header
        toks = ln.split()
        if not toks:
            continue
        vals = [int(t) for t in toks if t.lstrip("-").isdigit()]
        if vals:
            best = max(best, max(vals))
    return aln_a, aln_b, best


def main():
    if not os.path.isdir(REF):
        sys.exit("reference tree not present; fixtures are committed, nothing to do")
    os.makedirs(os.path.join(HERE, "queries"), exist_ok=True)

    recs = uniprot_dat_to_fasta(os.path.join(REF, "data/dbs/uniprot_subset.dat"))
    assert len(recs) == 111, len(recs)
    write_fasta(recs, os.path.join(HERE, "subset111.fasta"))

    for q in ("P01008", "P02232"):
        with open(os.path.join(REF, "test/reference/%s.txt" % q)) as f:
            lines = f.read().split("\n")
        scores = [ln for ln in lines if ln.strip()]
        with open(os.path.join(HERE, "%s.subset111.scores" % q), "w") as f:
            f.write("\n".join(scores[:111]) + "\n")
        with gzip.open(os.path.join(HERE, "%s.full.txt.gz" % q), "wt") as f:
            f.write("\n".join(scores) + "\n")

    for name in sorted(os.listdir(os.path.join(REF, "data/queries"))):
        shutil.copyfile(os.path.join(REF, "data/queries", name), os.path.join(HERE, "queries", name))

    binary = os.path.join(REPO, "oracle/_ref/cpu_ref")
    if not os.path.exists(binary):
        sys.exit("build oracle/_ref/cpu_ref first: make -C oracle ref")
    rng = random.Random(1782)
    pairs = [("HEAGAWGHEE", "PAWHEAE"), ("ACACACTA", "AGCACACA"),
             ("GGTTGACTA", "TGTTACGG"), ("A", "A"), ("A", "C"), ("MKV", "MKV")]
    amino = "ARNDCQEGHILKMFPSTWYV"
    for n in range(40):
        alpha = amino if n % 2 == 0 else "ACGT"
        la, lb = rng.randint(1, 300), rng.randint(1, 300)
        a = "".join(rng.choice(alpha) for _ in range(la))
        if n % 4 == 0:  # related pair: mutate a copy of a
            b = list(a[: lb])
            for k in range(len(b)):
                if rng.random() < 0.2:
                    b[k] = rng.choice(alpha)
            b = "".join(b) or "A"
        else:
            b = "".join(rng.choice(alpha) for _ in range(lb))
        pairs.append((a, b))
    out = []
    for a, b in pairs:
        aa, bb, best = cpu_ref_pair(binary, a, b)
        out.append({"a": a, "b": b, "aln_a": aa, "aln_b": bb, "max": best})
    with open(os.path.join(HERE, "cpu_pairs.json"), "w") as f:
        json.dump({"source": "oracle/_ref/cpu_ref built from /root/reference/src/cpu.cpp",
                   "scheme": {"match": 3, "mismatch": -3, "gap": 2}, "pairs": out}, f, indent=1)
    print("wrote fixtures to", HERE)


if __name__ == "__main__":
    main()
