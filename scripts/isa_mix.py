"""Instruction mix of one kernel's largest basic block (the unrolled
sub-group loop body) in a `hipcc --cuda-device-only -S` listing.
usage: isa_mix.py FILE.s SYMBOL_SUBSTRING"""
import collections
import re
import sys


def blocks(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and sym in l.split(":")[0])
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    cur, name = [], "entry"
    for l in lines[start + 1:end]:
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            yield name, cur
            cur, name = [], m.group(1)
            continue
        s = l.strip()
        if not s or s.startswith((";", ".", "//")):
            continue
        cur.append(s.split()[0])
    yield name, cur


if __name__ == "__main__":
    bl = list(blocks(sys.argv[1], sys.argv[2]))
    total = sum(len(b) for _, b in bl)
    name, big = max(bl, key=lambda x: len(x[1]))
    print(f"{sys.argv[2]}: {total} instructions, largest block {name}: {len(big)}")
    for k, v in collections.Counter(big).most_common(40):
        print(f"  {v:6d} {k}")
