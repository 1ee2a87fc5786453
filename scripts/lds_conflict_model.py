"""Expected LDS bank conflicts of the two-strips kernel's profile-image reads
on C2, from the guide's ds_read_b128 banking model
(/opt/skills/guides/MI355X_MICROARCH.md, LDS table): a wave's 64 lanes form
4 groups of 16, {0-3,12-15,20-27}, {4-11,16-19,28-31}, {32-35,44-47,52-59},
{36-43,48-51,60-63}; a lane's 16 bytes cover 4 banks, so a group's 16 lanes
cover the 64 banks as 16 slots of 16 bytes; lanes on the same address
broadcast, and a group costs one extra LDS cycle per extra distinct address
on its busiest slot (N-way = N cycles).

Each lane reads image row `code` (x2_row_dwords(32) = 36 dwords = 144 B = 9
slots per row, sw_inter_x2.hip), so lanes whose codes differ by a multiple of
16 (9 x 16 = 144 = 0 mod 16) share a slot with different addresses: A/T,
R/W, N/Y, D/V, I/pad, ...  With 26 possible codes and 16 slots per group
some pair always aliases, whatever the row stride (any odd stride aliases
exactly the codes equal mod 16), so the conflicts are inherent to b128 reads
of a code-indexed image; only which code pairs alias can change, by storing
the residues under a permuted code (`--perm`).

Every column's code vector is read 16 times per pass (8 ds_read_b128 per
32-row image, lo and hi), so the expected extra cycles per read is the mean
over columns of sum_g (max slot multiplicity - 1).

usage: python3 scripts/lds_conflict_model.py [--n 570000] [--sample 4000]
prints the model's extra cycles per ds_read_b128 for the code order as built
and for the frequency-aware permutation, beside the measured SQ ratio."""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ece1782-smith-waterman-cuda_amd"))
import synth  # noqa: E402

GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
          list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
          list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]
PAD = 25
ROW_SLOTS = 9  # 144-byte image rows (sw_inter_x2.hip x2_row_dwords(32) * 4 / 16)
# codes A R N D C Q E G H I L K M F P S T W Y V B J Z X * pad
NAMES = "ARNDCQEGHILKMFPSTWYVBJZX*_"


def extra_cycles(codes_by_lane, perm):
    """codes_by_lane: [ncols, 64] codes -> extra LDS cycles per read, per column."""
    phys = perm[codes_by_lane]
    slot_of = (np.arange(26) * ROW_SLOTS) % 16  # slot of each physical code
    total = np.zeros(codes_by_lane.shape[0], dtype=np.int64)
    for g in GROUPS:
        present = np.zeros((phys.shape[0], 26), dtype=np.int64)
        for lane in g:
            present[np.arange(phys.shape[0]), phys[:, lane]] = 1
        per_slot = np.zeros((phys.shape[0], 16), dtype=np.int64)
        for c in range(26):
            per_slot[:, slot_of[c]] += present[:, c]
        total += per_slot.max(axis=1) - 1
    return total


def frequency_perm():
    """Physical code of each code: slots 10..15 alone (16 slots, codes p and
    p + 16 share slot p * 9 mod 16) for the six most frequent residues, the
    pad's partner (physical 9) the next, the zero-frequency codes (B J Z X *)
    beside the next five, and the eight rarest standard residues paired
    rarest with most frequent."""
    f = dict(zip("ARNDCQEGHILKMFPSTWYV", synth.SWISSPROT_FREQ))
    std = sorted(f, key=lambda c: -f[c])
    phys = {}
    for k, c in enumerate(std[:6]):
        phys[c] = 10 + k
    phys[std[6]] = 9                       # shares with the pad (25)
    for k, (c, z) in enumerate(zip(std[7:12], "BJZX*")):
        phys[c] = k
        phys[z] = 16 + k
    rest = std[12:]                        # 8 rarest: pair rarest with most frequent
    for k in range(4):
        phys[rest[k]] = 5 + k
        phys[rest[-1 - k]] = 21 + k
    perm = np.array([phys[c] for c in NAMES[:25]] + [PAD], dtype=np.int64)
    assert sorted(perm.tolist()) == list(range(26))
    return perm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=570_000)
    ap.add_argument("--threshold", type=int, default=2048)
    ap.add_argument("--sample", type=int, default=3000, help="blocks sampled (cells-weighted)")
    ap.add_argument("--measured", type=float, default=9.34e8 / 3.22e8,
                    help="SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS of the profiled C2 launch")
    args = ap.parse_args()
    res, offs = synth.database(args.n, seed=synth.SEED, shard=0)
    L = np.diff(offs)
    order = np.argsort(-L, kind="stable")
    order = order[L[order] <= args.threshold]
    nblk = (len(order) + 63) // 64
    rng = np.random.default_rng(1)
    widths = np.array([L[order[64 * b]] for b in range(nblk)])
    pick = rng.choice(nblk, size=min(args.sample, nblk), replace=False, p=widths / widths.sum())
    ident = np.arange(26)
    perm = frequency_perm()
    tot_id = tot_pm = cols = 0
    for b in pick:
        subj = order[64 * b: 64 * b + 64]
        W = int(L[subj[0]])
        codes = np.full((W, 64), PAD, dtype=np.int64)
        for lane, s in enumerate(subj):
            codes[: L[s], lane] = res[offs[s]: offs[s + 1]]
        tot_id += extra_cycles(codes, ident).sum()
        tot_pm += extra_cycles(codes, perm).sum()
        cols += W
    print("blocks sampled %d (width-weighted), columns %d" % (len(pick), cols))
    print("model, codes as built: %.3f extra cycles per ds_read_b128" % (tot_id / cols))
    print("model, permuted codes: %.3f" % (tot_pm / cols))
    print("measured SQ ratio (all LDS instructions): %.3f" % args.measured)
    print("permutation (code -> physical):", {NAMES[c]: int(perm[c]) for c in range(26)})


if __name__ == "__main__":
    main()
