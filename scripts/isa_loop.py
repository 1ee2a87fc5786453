"""Per-iteration instruction counts of the sub-group loops of one kernel in a
`hipcc --cuda-device-only -S` listing (scripts/asm.sh): every loop whose body
holds more than 500 instructions, with its VALU / s_nop / LDS / VMEM counts
and the kernel's VGPR count.
usage: isa_loop.py FILE.s SYMBOL_SUBSTRING [SYMBOL_SUBSTRING ...]"""
import collections
import re
import sys


def kernel_lines(lines, sym):
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and sym in l.split(":")[0])
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    name = lines[start].split(":")[0]
    vgpr = None
    k = next((i for i, l in enumerate(lines) if l.strip() == ".amdhsa_kernel " + name), None)
    for l in lines[k:] if k is not None else []:
        m = re.search(r"\.amdhsa_next_free_vgpr (\d+)", l)
        if m:
            vgpr = int(m.group(1))
            break
    return name, lines[start + 1:end], vgpr


def loops(body):
    """Blocks grouped by their innermost loop header (asm comments)."""
    cur_hdr, out = None, collections.defaultdict(collections.Counter)
    for l in body:
        m = re.match(r"^(\.LBB\S+):\s*;(.*)$", l)
        if m:
            c = m.group(2)
            h = re.search(r"Header=(\S+)", c)
            cur_hdr = h.group(1) if h else ("BB" + m.group(1)[4:] if "Loop Header" in c else None)
            continue
        if re.match(r"^\.LBB\S+:", l):
            cur_hdr = None
            continue
        s = l.strip()
        if not s or s.startswith((";", ".", "//")) or cur_hdr is None:
            continue
        op = s.split()[0]
        k = out[cur_hdr]
        k["all"] += 1
        if op == "s_nop":
            k["s_nop"] += 1
        elif op.startswith("v_"):
            k["valu"] += 1
            if op.startswith("v_pk_"):
                k["v_pk"] += 1
        elif op.startswith("ds_"):
            k["lds"] += 1
        elif op.startswith(("global_", "buffer_")):
            k["vmem"] += 1
        elif op == "s_barrier":
            k["barrier"] += 1
    return out


if __name__ == "__main__":
    lines = open(sys.argv[1]).read().split("\n")
    for sym in sys.argv[2:]:
        name, body, vgpr = kernel_lines(lines, sym)
        print(f"{sym}  vgpr={vgpr}")
        for hdr, k in loops(body).items():
            if k["all"] > int(__import__("os").environ.get("MINLOOP", "500")):
                print(f"  loop {hdr}: " + " ".join(f"{n}={k[n]}" for n in ("all", "valu", "v_pk", "s_nop", "lds", "vmem", "barrier")))
