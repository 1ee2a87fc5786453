#!/usr/bin/env python3
"""bench.py — headline measurement of the Smith-Waterman database scan.

Default workload (BASELINE.json configs[1]): the
375-residue query P07327 (data/queries/P07327.fasta of the reference, shipped
as a fixture) against a Swiss-Prot-sized synthetic database (570,000
subjects, log-normal lengths median 290 / mean ~360, Swiss-Prot residue
frequencies; Swiss-Prot itself is not available here), scored as configs[1]
states: BLOSUM62 with affine gaps, BLAST's default 11/1 (a gap of k residues
costs 11 + k, i.e. gap_open 12 and gap_extend 1 in this library's
convention).  The reference's own scoring (BLOSUM50 of SWSolver.cu:54-81,
linear gap 2) is timed the same way right after and reported under
"reference_scoring".

--config c3: the 20 shipped queries (144..5478 aa, sum 41,752) as one batch
against the same database (configs[2]); --config c4: P07327 against a
50,000,000-subject database split over the ranks by id range (configs[3]),
each rank's shard generated in its GPU's HBM from (seed, global id) by the
counter-based generator (sw_db_create_synthetic); --config c5: a
5,000-residue synthetic query against 10,000 subjects of N(2000, 200)
residues (configs[4]); --config c1: P02232 (144 aa) against 1,000 synthetic
subjects on the CPU restatement of cpu.cpp's recurrence at one thread and at
every host core, the literal cpu.cpp beside it (configs[0]; no GPU timing in
`value`).

One step = one pass of the hot path over the rank's resident shard: build the
query profile(s), run the scan kernels (intra-sequence for subjects longer
than the long threshold, inter-sequence for the rest), then the top-K
exchange (device top-K per query, RCCL all-gather of K (score, global id)
keys per rank, device merge).

Multi-GPU (torchrun, one process per GPU) is STRONG scaling: every rank
builds the same database and scans only its residue-balanced share (LPT over
subject lengths, dist.shard_indices; C4: an id range), so N GPUs search one
database of fixed size.  value = all cells of the database / the max-over-
ranks time of K steps.  After timing, every rank re-scores its share with
the CPU oracle (all of it when that fits --verify-seconds, else a random
sample plus its top-K hits), checks its device top-K against a CPU top-K of
its scores, and rank 0 checks the RCCL-merged top-K against the merge of
the oracle's per-rank top-K (the bit-exact top-score list of north_star);
--shard-of N --shard-rank R measures rank R's share of N GPUs on one GPU.

Prints ONE JSON line on rank 0.
"""
import argparse
import hashlib
import json
import math
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "GCUPS (DP cell updates/s) query-vs-SwissProt, 1/2/4/8 MI355X; bit-exact scores"
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SIMDS, CLOCK_HZ = 1024, 2.4e9   # 256 CUs x 4 SIMDs
# VALU issue model of each per-wave inter kernel: SIMD cycles per DP cell,
# from the compiled inner loop's instruction counts (hipcc -S) priced at the
# measured gfx950 issue costs (profiles/r01_valu_rate_*.txt: v_sub_u32 clamp
# 2.45, v_max_i32 4.37, v_max3_i32 4.4, v_add_u32_sdwa 4.2, v_pk_* 4.25
# (v_pk_maximum3_f16 and v_pk_add_f16 too, profiles/r01_f16_rate.txt),
# v_or_b32 2.7 cycles per wave64 instruction).
VALU_MODEL = {
    # per 2 x 64 cells: every VALU instruction of the sub-group loop (hipcc -S,
    # the blocks of one 8-column sub-group = 256 cell pairs): the biased fp16
    # cell (5 packed ops + ~0.53 v_pk_maximum3_f16 for the anti-diagonal
    # maxima + column rebase + row-group resets) = 5.91 packed, 0.38 other
    "sw_inter_x2s<32,8,affine,fp16>": (5.91 * 4.25 + 0.305 * 2.7) / 128,
    # linear int16: 2.81 v_pk_max_i16, 0.94 v_pk_sub_u16, 0.94 v_pk_mad_u16
    # in the hot block, 5.0 packed + 0.29 other over the whole loop
    "sw_inter_x2s<32,8,linear>": (5.0 * 4.25 + 0.29 * 2.7) / 128,
    # the biased linear fp16 cell: fma, max3, floor max + ~0.53 maxima = 3.73
    # packed, 0.32 other
    "sw_inter_x2s<32,8,linear,fp16>": (3.86 * 4.25 + 0.305 * 2.7) / 128,
    "sw_inter_x2p<32,8,linear,fp16>": (3.86 * 4.25 + 0.305 * 2.7) / 128,
    # (the merged launch's 48-row strips under linear gaps: the same cell)
    "sw_inter_x2p<48,8,linear,fp16>": (3.86 * 4.25 + 0.305 * 2.7) / 128,
    # the same cells with the widest blocks run by wave pairs in the same launch
    "sw_inter_x2p<32,8,affine,fp16>": (5.91 * 4.25 + 0.305 * 2.7) / 128,
    "sw_inter_x2p<32,8,linear>": (5.0 * 4.25 + 0.29 * 2.7) / 128,
    # per 2 x 64 cells: 4.53 v_pk_max_i16, 2.65 v_pk_sub_u16, 0.94 v_pk_mad_u16
    "sw_inter_x2p<32,8,affine>": (8.117 * 4.25) / 128,
    "sw_inter_x2s<32,8,affine>": (8.117 * 4.25) / 128,
    # per 64 cells: 1.5 v_max3, 1 v_add_sdwa, 1 v_sub clamp
    "sw_inter<64,8,linear>": (1.5 * 4.4 + 4.2 + 2.45) / 64,
    # per 64 cells: 2.82 v_sub clamp, 1.83 v_max, 1.5 v_max3, 1 v_add_sdwa
    "sw_inter<32,8,affine>": (2.82 * 2.45 + 1.83 * 4.37 + 1.5 * 4.4 + 4.2) / 64,
}
# sw_intra_x2<RI> (two long subjects per wave, the biased fp16 cell): per
# lane-step, RI rows x (1 v_perm_b32 + 1 v_pk_add_f16 for H_diag + S, 5
# packed cell ops incl. E's max, 0.53 v_pk_maximum3_f16 for the anti-diagonal
# maxima, 0.25 for the rebase every 8 steps) for 2 x 64 cells, plus ~80
# cycles of conveyor work (3 DPP moves, 3 readlanes, 2 hand-off adjusts, the
# profile addresses, lane 63's boundary store; hipcc -S of sw_intra_x2.hip;
# SQ_INSTS_VALU on C5 at RI = 16: 130 per lane-step, profiles/r02_sq/)
for _ri in (4, 6, 8, 10, 12, 16, 20):
    VALU_MODEL["sw_intra_x2<%d>" % _ri] = (_ri * (6.78 * 4.25) + 80.0) / (128 * _ri)
MATRICES = {"blosum50": 0, "blosum62": 1}
SEED = 1782
C4_TOTAL = 50_000_000
C3_QUERIES = ["P02232", "P05013", "P14942", "P07327", "P01008", "P03435", "P42357", "P21177",
              "Q38941", "P27895", "P07756", "P04775", "P19096", "P28167", "P0C6B8", "P20930",
              "P08519", "Q7TMA5", "P33450", "Q9UKN1"]
# sources whose change can change the dominant kernel's HBM traffic: a stored
# rocprofv3 --pmc measurement (pmc_traffic.json) is only reported for the
# build it was taken on
KERNEL_SOURCES = ["sw_inter_x2.hip", "sw_intra_x2.hip", "sw_intra_x2.h", "sw_int32.h", "sw_kernels.hip", "sw_kernels.h", "sw_capi.cpp", "sw_plan.cpp"]


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def read_query(name):
    with open(os.path.join(REPO, "tests", "golden", "queries", name + ".fasta")) as f:
        return "".join(f.read().split("\n")[1:])


def kernel_source_hash():
    h = hashlib.sha256()
    for name in KERNEL_SOURCES:
        with open(os.path.join(REPO, "ece1782-smith-waterman-cuda_amd", "csrc", name), "rb") as f:
            h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def workload_key(args, qlen):
    key = "%s/%d/%d/%s-%d-%d" % (args.query, args.db_seqs, qlen, args.matrix, args.gap_open, args.gap_extend)
    return key if args.config == "c2" else args.config + ":" + key


def traffic_entry(tj, key):
    """The stored PMC measurement of a workload: pmc_traffic.json holds the
    headline (C2) entry at its top level and every measured workload under
    "workloads" (scripts/pmc_traffic.py --merge)."""
    if tj.get("workload_key") == key:
        return tj
    return tj.get("workloads", {}).get(key)


def host_cores():
    """(cores this process may use, logical CPUs in its affinity mask, the
    cgroup CPU quota in cores or None).  GPU boxes show the whole host's CPUs
    in the mask; the quota is the share actually granted."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                p = int(f.read())
            if q > 0:
                quota = q / p
        except (OSError, ValueError):
            pass
    eff = aff if quota is None else max(1, min(aff, int(math.ceil(quota))))
    return eff, aff, quota


# The algorithm's VALU floor: packed 16-bit ops per cell PAIR
# (two cells per instruction) of the biased cell, without the maxima, the
# rebase or any addressing — affine (Gotoh): v_pk_fma (H_diag + S),
# v_pk_maximum3 (H), v_pk_add (H - open), v_pk_maximum (E), v_pk_maximum3
# (F with the floor); linear: v_pk_fma, v_pk_maximum3, v_pk_maximum (floor).
# Each packed op issues in 4.25 SIMD cycles on gfx950
# (profiles/r01_f16_rate.txt).
FLOOR_PACKED_OPS = {True: 5, False: 3}
PACKED_OP_CYCLES = 4.25


def algorithmic_peak_gcups(affine, clock_ghz):
    """1,024 SIMDs x clock / (floor packed ops x 4.25 cycles) x 128 cells
    (a wave64 packed op updates 2 x 64 cells)."""
    return SIMDS * clock_ghz * 1e9 / (FLOOR_PACKED_OPS[affine] * PACKED_OP_CYCLES) * 128 / 1e9


def valu_roofline(kernel, cells_rank, scan_ms, kernel_gcups, affine, clock_load_ghz=None):
    """The binding roofline: VALU instruction issue.  achieved = the whole
    scan's rate (all kernels of the scan, concurrent).
    `algorithmic`: peak = the algorithm's floor of packed ops per cell pair
    (FLOOR_PACKED_OPS) at 4.25 cycles each on every SIMD, at the 2.4 GHz
    peak clock and at the clock measured under this load (the stored SQ
    pass, when it is of this build): the distance of the scan from the
    algorithm, every instruction the kernels add counted against them.
    `issue_efficiency`: peak = the rate the kernel's OWN compiled
    instruction mix allows (VALU_MODEL, hipcc -S counts); its frac measures
    how well the code as written issues, not how far it is from the floor."""
    if scan_ms <= 0:
        return None
    achieved = cells_rank / (scan_ms * 1e-3) / 1e9
    peak = algorithmic_peak_gcups(affine, CLOCK_HZ / 1e9)
    alg = {"floor_packed_ops_per_cell_pair": FLOOR_PACKED_OPS[affine], "cycles_per_packed_op": PACKED_OP_CYCLES,
           "simds": SIMDS, "clock_ghz": CLOCK_HZ / 1e9, "peak": round(peak, 1), "frac": round(achieved / peak, 4),
           "clock_ghz_under_load": clock_load_ghz, "peak_under_load": None, "frac_under_load": None}
    if clock_load_ghz:
        pl = algorithmic_peak_gcups(affine, clock_load_ghz)
        alg["peak_under_load"] = round(pl, 1)
        alg["frac_under_load"] = round(achieved / pl, 4)
    out = {"bound": "valu-issue", "achieved": round(achieved, 1), "peak": alg["peak"], "unit": "GCUPS",
           "frac": alg["frac"], "kernel": kernel, "algorithmic": alg,
           "kernel_alone_gcups_while_concurrent": round(kernel_gcups, 1)}
    cpc = VALU_MODEL.get(kernel.split("+")[0])  # "+int16[0,n)": the widest blocks in int16 beside it
    if cpc is not None:
        ip = SIMDS * CLOCK_HZ / cpc / 1e9
        out["issue_efficiency"] = {"peak": round(ip, 1), "frac": round(achieved / ip, 4),
                                   "simd_cycles_per_cell": round(cpc, 5),
                                   "note": "peak from the kernel's own compiled instruction mix (VALU_MODEL): "
                                           "issue efficiency of the code as written, not a roofline"}
    return out


def reference_scoring_summary(elapsed_s, cells_all, steps, kt, kernels, cold_ms, parity, parity_ok):
    """The `reference_scoring` object: the same step timed under the
    reference's own scoring (BLOSUM50 of SWSolver.cu:54-81, linear gap 2 of
    :7), with the parity of its last step's scores against the oracle."""
    n = max(kt["scans"], 1)
    out = {"scoring": "BLOSUM50 (SWSolver.cu:54-81), linear gap 2 (the reference's own)",
           "value": round(cells_all * steps / elapsed_s / 1e9, 2), "unit": "GCUPS",
           "ms_per_step": round(elapsed_s * 1e3 / steps, 3), "kernel": kernels[0], "intra_kernel": kernels[1],
           "kernel_ms_per_scan": {"sw_inter": round(kt["wave_ms"] / n, 4),
                                  "sw_inter_coop": round(kt["coop_ms"] / n, 4),
                                  "sw_intra": round(kt["intra_ms"] / n, 4),
                                  "scan_total": round(kt["total_ms"] / n, 4)},
           "cold_first_scan_ms": cold_ms}
    if parity is not None:
        out["parity"] = parity
        out["parity_ok"] = parity_ok
    return out


def host_sampler(res, offs):
    """Subjects idx of a host-resident shard as (residues, offsets)."""
    def take(idx):
        idx = np.asarray(idx, dtype=np.int64)
        if len(idx) == len(offs) - 1:
            return res, offs
        lens = offs[idx + 1] - offs[idx]
        so = np.zeros(len(idx) + 1, dtype=np.int64)
        so[1:] = np.cumsum(lens)
        sr = np.concatenate([res[offs[i]:offs[i + 1]] for i in idx]) if len(idx) else np.zeros(0, np.uint8)
        return sr, so
    return take


def counter_sampler(sw, seed, id_base):
    """Subjects idx of a device-generated shard, regenerated on the CPU by
    the counter-based restatement (synth.counter_*)."""
    L, lut = sw.capi.synth_tables()

    def take(idx):
        gids = id_base + np.asarray(idx, dtype=np.int64)
        lens = sw.synth.counter_lengths(seed, gids, L)
        so = np.zeros(len(idx) + 1, dtype=np.int64)
        so[1:] = np.cumsum(lens)
        sr = np.concatenate([sw.synth.counter_residues(seed, int(g), int(m), lut) for g, m in zip(gids, lens)]) \
            if len(idx) else np.zeros(0, np.uint8)
        return sr, so
    return take


def oracle_scan(queries, sr, so, scoring, threads):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import sw_oracle
    mat, go, ge = scoring
    return [sw_oracle.scan(q, sr, so, mat=mat, gap_open=go, gap_extend=ge, nthreads=threads) for q in queries]


def cpu_baseline(queries, sampler, n, gpu_scores, seconds, threads, scoring, one_thread_seconds):
    """The oracle (C restatement of cpu.cpp's recurrence, Gotoh for affine;
    kind "port") on a bounded random sample of the same shard, every query of
    the workload, with the same scoring as the GPU run: at `threads` threads
    (the cores this process may use) and at one thread.  sampler(idx) ->
    (residues, offsets) of shard subjects idx; gpu_scores: [nq][n] scores of
    the measured run (parity check of the sample)."""
    rng = np.random.default_rng(1782)
    perm = rng.permutation(n)
    qtot = sum(len(q) for q in queries)

    def timed(m, nt):
        idx = np.sort(perm[:m])
        sr, so = sampler(idx)
        t = time.perf_counter()
        out = oracle_scan(queries, sr, so, scoring, nt)
        return idx, so, out, time.perf_counter() - t

    def sized(nt, budget):
        # calibrate on growing samples until one takes >= 0.3 s (thread
        # start-up dominates tiny samples), then size the real one to budget
        m0 = min(n, 50)
        while True:
            idx, so, out, dt = timed(m0, nt)
            if dt >= 0.3 or m0 >= n:
                break
            m0 = min(n, m0 * 4)
        m = int(min(n, max(m0, m0 * budget / max(dt, 1e-3))))
        return timed(m, nt) if m != m0 else (idx, so, out, dt)

    idx, so, cpu, dt = sized(threads, seconds)
    cells = qtot * int(so[-1])
    parity = all(bool(np.array_equal(c, gpu_scores[k][idx])) for k, c in enumerate(cpu))
    idx1, so1, cpu1, dt1 = sized(1, one_thread_seconds)
    cells1 = qtot * int(so1[-1])
    parity = parity and all(bool(np.array_equal(c, gpu_scores[k][idx1])) for k, c in enumerate(cpu1))
    return {"value": round(cells / dt / 1e9, 4), "unit": "GCUPS", "cores": threads, "kind": "port",
            "one_thread": round(cells1 / dt1 / 1e9, 4),
            "sample": "%d of %d subjects (%d residues) of rank 0's shard x %d quer%s (%d residues), %.3g cells, "
                      "%.1f s on %d threads; one thread: %d subjects, %.3g cells, %.1f s; scores equal to the "
                      "GPU's: %s" % (len(idx), n, int(so[-1]), len(queries), "y" if len(queries) == 1 else "ies",
                                     qtot, cells, dt, threads, len(idx1), cells1, dt1, parity)}, parity


def verify(sw, dist, world, rank, queries, sampler, n, gids, gpu_scores, dev_top, final, K, scoring, threads,
           seconds, backend):
    """Parity of the measured run at any N (outside the timed region).

    Every rank: (1) its device top-K == a CPU top-K of its GPU scores (global
    ids, score desc / id asc); (2) the oracle re-scores its share (all of it
    if the estimate fits `seconds`, else a random sample) and every score must
    be equal; its top-K hits are re-scored too.  Rank 0: (3) when every rank
    scored its whole share, the RCCL-merged top-K must equal the merge of the
    per-rank ORACLE top-K (the bit-exact top-score list); otherwise the merge
    of the per-rank CPU top-K of the GPU scores."""
    nq = len(queries)
    qtot = sum(len(q) for q in queries)
    # the device top-K is always K long, padded with INT64_MIN past a short share
    ok_topk = all(np.array_equal(dev_top[k], _pad_keys(sw.dist.local_topk(gpu_scores[k], gids, K), K))
                  for k in range(nq))
    # the rank's top-K hits (local indices) are always re-scored
    pos = {int(g): i for i, g in enumerate(gids)} if len(gids) else {}
    hit_local = set()
    for k in range(nq):
        ids, _ = sw.capi.decode_keys(dev_top[k])
        hit_local.update(pos[int(g)] for g in ids if g >= 0)
    # estimate the oracle's rate from a calibration sample grown until it
    # takes >= 0.5 s (thread start-up dominates tiny samples and made the
    # estimate ~2x low: whole shares that fit the budget were only sampled)
    rng = np.random.default_rng(1782 + rank)
    perm = rng.permutation(n)
    m0 = min(n, 256)
    while True:
        cal = np.sort(perm[:m0])
        sr, so = sampler(cal)
        t = time.perf_counter()
        oracle_scan(queries, sr, so, scoring, threads)
        dt_cal = time.perf_counter() - t
        if dt_cal >= 0.5 or m0 >= n:
            break
        m0 = min(n, m0 * 4)
    rate = qtot * int(so[-1]) / max(dt_cal, 1e-4)
    res_total = None
    try:
        _, offs = sampler.full
        res_total = int(offs[-1])
    except AttributeError:
        pass
    full = res_total is not None and qtot * res_total / rate <= seconds
    if full:
        idx = np.arange(n)
    else:
        m = int(min(n, max(m0, m0 * seconds / max(qtot * int(so[-1]) / rate, 1e-4))))
        idx = np.unique(np.concatenate([perm[:m], np.fromiter(hit_local, dtype=np.int64, count=len(hit_local))]))
    sr, so = sampler(idx)
    t = time.perf_counter()
    cpu = oracle_scan(queries, sr, so, scoring, threads)
    dt = time.perf_counter() - t
    ok_scores = all(bool(np.array_equal(c, gpu_scores[k][idx])) for k, c in enumerate(cpu))
    # per-rank top-K keys: of the oracle's scores (whole share) or of the GPU's
    src = cpu if full else gpu_scores
    sel = gids[idx] if full else gids
    mine = np.stack([_pad_keys(sw.dist.local_topk(src[k], sel, K), K) for k in range(nq)])
    checked = np.array([len(idx), n, int(full), int(ok_topk), int(ok_scores)], dtype=np.int64)
    if world > 1:
        allkeys = dist.allgather_np(mine)
        allchk = dist.allgather_np(checked)
    else:
        allkeys = mine[None]
        allchk = checked[None]
    merged_ok = all(np.array_equal(sw.dist.merge_topk([allkeys[r][k] for r in range(world)], K),
                                   final[k][final[k] != np.iinfo(np.int64).min]) for k in range(nq))
    all_full = bool(allchk[:, 2].all())
    res = {"subjects_checked": int(allchk[:, 0].sum()), "subjects": int(allchk[:, 1].sum()),
           "whole_database": all_full,
           "rank_topk_equal_cpu_topk": bool(allchk[:, 3].all()),
           "scores_equal_oracle": bool(allchk[:, 4].all()),
           "merged_topk_equal": merged_ok,
           "merged_topk_reference": ("merge of the per-rank oracle top-%d (every subject re-scored)" % K)
           if all_full else ("merge of the per-rank CPU top-%d of the GPU scores (oracle sample)" % K),
           "oracle_threads_per_rank": threads, "oracle_seconds_rank0": round(dt, 2),
           "cells_checked_rank0": float(qtot * int(so[-1]))}
    ok = res["rank_topk_equal_cpu_topk"] and res["scores_equal_oracle"] and merged_ok
    return res, ok


def _pad_keys(keys, K):
    out = np.full(K, np.iinfo(np.int64).min, dtype=np.int64)
    out[:len(keys)] = keys[:K]
    return out


def c1_main(args):
    """configs[0]: P02232 (144 aa) vs 1,000 synthetic subjects on the CPU
    reference path — the oracle at one thread and at every core this process
    may use, the literal cpu.cpp (oracle/_ref/cpu_ref, +/-3 scoring, prints
    its matrices) on a few pairs beside it, and the GPU on the same database
    for comparison.  value = the oracle at all cores (the reference path)."""
    import _swpkg
    sw = _swpkg.load()
    eff, aff, quota = host_cores()
    threads = args.cpu_threads or eff
    q = sw.encode(read_query("P02232"))
    res, offs = sw.synth.database(args.db_seqs or 1000, shard=0)
    n = len(offs) - 1
    scoring = (sw.capi.builtin_matrix(0), 2, 2)
    cells = float(len(q)) * int(offs[-1])

    def rate(nt, reps):
        best = 1e30
        for _ in range(reps):
            t = time.perf_counter()
            out = oracle_scan([q], res, offs, scoring, nt)[0]
            best = min(best, time.perf_counter() - t)
        return out, cells / best / 1e9, best

    want, r1, t1 = rate(1, 3)
    _, rall, tall = rate(threads, 5)
    out = {"metric": METRIC, "value": round(rall, 3), "unit": "GCUPS", "n_gpus": 0, "steps": 5, "warmup": 0,
           "ms_per_step": round(tall * 1e3, 3), "higher_is_better": True, "scaling": "none",
           "vs_baseline": None, "dtype": "int32", "data": "synthetic",
           "config": {"workload": "C1: P02232 (144 aa) vs %d synthetic subjects (%d residues), BLOSUM50 "
                                  "(SWSolver.cu:54-81) linear gap 2, CPU restatement of cpu.cpp:43-74" % (n, offs[-1]),
                      "config": "c1", "cells": cells},
           "cpu_baseline": {"value": round(rall, 3), "unit": "GCUPS", "cores": threads, "kind": "port",
                            "one_thread": round(r1, 4),
                            "sample": "the whole C1 database, best of 5 runs at %d threads, best of 3 at one "
                                      "thread" % threads},
           "host": {"cores_used": threads, "affinity_cpus": aff, "cgroup_quota_cpus": quota}}
    ref = os.path.join(REPO, "oracle", "_ref", "cpu_ref")
    if os.path.exists(ref):
        # the literal cpu.cpp: one pair per process, +/-3 scoring, prints
        # its alignment and both matrices (to /dev/null here)
        letters = "ARNDCQEGHILKMFPSTWYVBJZX*"
        qs = "".join(letters[c] for c in q)
        npairs = min(n, 40)
        c = 0
        t = time.perf_counter()
        for k in range(npairs):
            s = "".join(letters[x] for x in res[offs[k]:offs[k + 1]])
            subprocess.run([ref, qs, s], stdout=subprocess.DEVNULL, check=True)
            c += len(q) * len(s)
        dt = time.perf_counter() - t
        out["reference_cpu_cpp"] = {"value": round(c / dt / 1e9, 5), "unit": "GCUPS", "cores": 1,
                                    "kind": "reference",
                                    "sample": "oracle/_ref/cpu_ref (built from the untouched cpu.cpp) on the first "
                                              "%d pairs, +/-3 scoring as cpu.cpp hard-codes, one process per pair "
                                              "printing its matrices to /dev/null: %.3g cells in %.2f s" % (npairs, c, dt)}
    if not args.no_gpu:
        h = sw.Handle(0)
        db = sw.Database(h, res, offs)
        got = db.scan(q, *scoring)
        best = 1e30
        for _ in range(5):
            t = time.perf_counter()
            db.scan(q, *scoring)
            best = min(best, time.perf_counter() - t)
        out["gpu_same_workload"] = {"value": round(cells / best / 1e9, 2), "unit": "GCUPS",
                                    "note": "synchronous sw_scan incl. profile upload and D2H of %d scores, "
                                            "best of 5 (latency-bound at this size)" % n}
        out["parity_sample_ok"] = bool(np.array_equal(got, want))
        db.close()
        h.close()
    print(json.dumps(out), flush=True)


def make_workload(sw, args, world, rank):
    """(queries, query names, residues, offsets, global ids, description, full
    database) for this rank's share of ONE database."""
    if args.config == "c4":
        return [sw.encode(read_query(args.query))], [args.query], None, None, None, \
            "C4: query %s (%d aa) vs a %d-subject synthetic db generated on the devices" % (
                args.query, len(read_query(args.query)), C4_TOTAL), None
    if args.config in ("c2", "c3"):
        res, offs = sw.synth.database(args.db_seqs, shard=0)
    else:  # c5: one 5,000-residue query vs 10,000 subjects of N(2000, 200)
        res, offs = sw.synth.fixed_length_database(args.db_seqs, 2000, 200, shard=0)
    gids, r_res, r_offs = sw.dist.shard(res, offs, rank, world)
    if args.config == "c2":
        qs, names = [sw.encode(read_query(args.query))], [args.query]
        desc = "C2: query %s (%d aa) vs synthetic Swiss-Prot-sized db" % (args.query, len(qs[0]))
    elif args.config == "c3":
        qs, names = [sw.encode(read_query(n)) for n in C3_QUERIES], C3_QUERIES
        desc = "C3: batch of the %d shipped queries (%d..%d aa, sum %d) vs synthetic Swiss-Prot-sized db" % (
            len(qs), min(map(len, qs)), max(map(len, qs)), sum(map(len, qs)))
    else:
        qs, names = [sw.synth.query(5000)], ["synthetic-5000"]
        desc = "C5: synthetic 5000-aa query vs N(2000, 200)-residue subjects"
    return qs, names, r_res, r_offs, gids, desc, (res, offs)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, attempts=2):
    """`bench.py --gpus N` started without a torchrun environment: start N
    ranks as ONE child process (`python -m torch.distributed.run`, one rank per
    GPU, rendezvous on 127.0.0.1), relay rank 0's single JSON line and return
    the child's exit code.  Runs before anything in this process touches HIP
    (torch is not even imported here) and never replaces this process.  The
    rendezvous port is picked free just before the launch; if another process
    takes it in between (the child fails with no JSON line and an address-in-
    use error), the launch is tried once more on a new port."""
    for attempt in range(attempts):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
        log("starting %d ranks: %s" % (n, " ".join(cmd)))
        proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, cwd=REPO)
        lines, port_taken = [], False
        for line in proc.stdout:
            s = line.strip()
            if s.startswith("{") and '"metric"' in s:
                lines.append(s)
            elif s:
                port_taken = port_taken or "address already in use" in s.lower() or "EADDRINUSE" in s
                print(s, file=sys.stderr, flush=True)
        rc = proc.wait()
        if rc != 0 and not lines and port_taken and attempt + 1 < attempts:
            log("rendezvous port taken; retrying on another port")
            continue
        break
    if rc == 0 and len(lines) != 1:
        log("expected one JSON line from rank 0, got %d" % len(lines))
        rc = 1
    if lines:
        print(lines[-1], flush=True)
    return rc


def sustained_summary(elapsed_s, steps, cells_per_step, kernel_ms_total, nscans, world):
    """The `sustained` object: back-to-back steps for >= --sustained-seconds
    after the timed region (not part of `value`), so clock droop under
    continuous load shows, with the scan kernel's HIP-event time beside it."""
    return {"seconds": round(elapsed_s, 3), "steps": steps, "n_gpus": world,
            "value": round(cells_per_step * steps / elapsed_s / 1e9, 2), "unit": "GCUPS",
            "ms_per_step": round(elapsed_s * 1e3 / steps, 4),
            "kernel_ms_per_scan": round(kernel_ms_total / max(nscans, 1), 4),
            "note": "outside value: the same step back to back for the stated seconds after the timed region "
                    "(max over ranks), scan kernel time from the library's HIP events"}


def check_world(gpus, env):
    """Return the WORLD_SIZE to run with, or raise SystemExit when it
    disagrees with --gpus (a silent one-rank measurement would be reported as
    an N-GPU number)."""
    world = int(env.get("WORLD_SIZE", "1"))
    if world != gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE %d: refusing to measure a different number of ranks "
                         "than asked (start without WORLD_SIZE to let bench.py launch the ranks)" % (gpus, world))
    return world


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c4", "c5"],
                    help="c2 = the headline (BASELINE configs[1]); c1 / c3 / c4 / c5 = configs[0] / [2] / [3] / [4]")
    ap.add_argument("--steps", type=int, default=None, help="default 100 (c2, c5) / 3 (c3, c4)")
    ap.add_argument("--warmup", type=int, default=None, help="default 20 (c2, c5) / 1 (c3, c4)")
    ap.add_argument("--db-seqs", type=int, default=None,
                    help="subjects of the WHOLE database (default 570000; c1: 1000; c4: 50M; c5: 10000)")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="measure one rank's share of this many GPUs on this GPU (strong-scaling rehearsal)")
    ap.add_argument("--shard-rank", type=int, default=0)
    ap.add_argument("--rehearse-exchange", action="store_true",
                    help="with --shard-of N: each step also runs the N-rank exchange's device work on the "
                         "exchange stream: a one-rank RCCL all-gather of the top-K, the other N-1 rows "
                         "copied in, and the device merge of N x K keys")
    ap.add_argument("--query", default="P07327")
    ap.add_argument("--topk", type=int, default=100)
    ap.add_argument("--matrix", default="blosum62", choices=sorted(MATRICES))
    ap.add_argument("--gap-open", type=int, default=12, help="cost of a 1-residue gap (BLAST 11/1 -> 12)")
    ap.add_argument("--gap-extend", type=int, default=1)
    ap.add_argument("--no-reference-scoring", action="store_true",
                    help="skip the second timed loop with the reference's BLOSUM50 / linear 2")
    ap.add_argument("--long-threshold", type=int, default=0, help="0 = library default")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core this process may use")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify-seconds", type=float, default=25.0,
                    help="oracle budget per rank for the parity leg (whole share if it fits)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-gpu", action="store_true", help="c1: skip the GPU comparison")
    ap.add_argument("--no-overlap", action="store_true",
                    help="run each step's top-K exchange on the scan's stream instead of overlapping the next scan")
    # high priority: HIP gives such streams their own hardware queues, so the
    # exchange never shares one (in order) with the scan's main, long-subject
    # or int16 side streams (GPU_MAX_HW_QUEUES = 4 normal-priority queues)
    ap.add_argument("--exchange-priority", type=int, default=-1,
                    help="HIP stream priority of the exchange stream (negative = higher)")
    # the latest rocprofv3 --pmc measurement of the C2 launch (FETCH_SIZE x2 +
    # WRITE_SIZE, scripts/pmc_traffic.py); kept at the root because profiles/
    # does not travel to the GPU box
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "pmc_traffic.json"))
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo = rehearse the multi-rank path on one GPU (CPU collectives)")
    ap.add_argument("--device", type=int, default=None, help="override the GPU index (rehearsal)")
    ap.add_argument("--sustained-seconds", type=float, default=5.0,
                    help="after the timed steps, run the step back to back this long and report it as "
                         "`sustained` (outside value; 0 = skip)")
    args = ap.parse_args()
    if args.config == "c1":
        return c1_main(args)
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if args.shard_of:
            raise SystemExit("--shard-of is a one-process rehearsal")
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.rehearse_exchange and not args.shard_of:
        raise SystemExit("--rehearse-exchange needs --shard-of")
    if args.steps is None:
        args.steps = 3 if args.config in ("c3", "c4") else 100
    if args.warmup is None:
        # 20 short steps (a 1/8 share's step is ~1.3 ms): the first ~0.1 s of
        # back-to-back scans on a GPU that was idle ran up to 5 % slower
        # (scripts/gpu_r02_thr.sh, the first of two identical runs)
        args.warmup = 1 if args.config in ("c3", "c4") else 20
    if args.db_seqs is None:
        args.db_seqs = {"c5": 10000, "c4": C4_TOTAL}.get(args.config, 570000)

    import torch
    import torch.distributed as tdist

    world = check_world(args.gpus, os.environ)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    # the database is split over shard_world ranks; this process scans share
    # shard_rank (= its rank, or the rehearsed one with --shard-of)
    shard_world, shard_rank = (args.shard_of, args.shard_rank) if args.shard_of else (world, rank)
    if args.shard_of and world > 1:
        raise SystemExit("--shard-of is a one-process rehearsal")
    gpu = local if args.device is None else args.device
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if args.backend == "nccl":
            tdist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            tdist.init_process_group("gloo", rank=rank, world_size=world)
    elif args.rehearse_exchange:
        # a one-rank RCCL communicator: the all-gather's launch and kernel on
        # the exchange stream (the peers' transfers are not rehearsed)
        tdist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0,
                                 world_size=1, device_id=dev)

    import _swpkg
    sw = _swpkg.load()

    t0 = time.perf_counter()
    queries, qnames, res, offs, gids, desc, full_db = make_workload(sw, args, shard_world, shard_rank)
    nq = len(queries)
    qtot = sum(len(q) for q in queries)

    handle = sw.Handle(gpu)
    # The library launches on a torch stream (not the legacy null stream,
    # whose handle is 0 = "library-owned stream" for sw_set_stream), so the
    # scan is stream-ordered with the top-K ops that read its scores.
    stream = torch.cuda.Stream(dev)
    handle.set_stream(stream.cuda_stream)
    torch.cuda.set_stream(stream)
    if res is None:  # c4: an id range of the database, generated in this GPU's HBM
        per = -(-args.db_seqs // shard_world)
        id_base = shard_rank * per
        n_mine = max(0, min(per, args.db_seqs - id_base))
        db = sw.Database.synthetic(handle, SEED, n_mine, id_base=id_base,
                                   long_threshold=(args.long_threshold or None))
        lens, _ = db.subjects()
        offs = np.zeros(len(lens) + 1, dtype=np.int64)
        offs[1:] = np.cumsum(lens)
        sampler = counter_sampler(sw, SEED, id_base)
        gids = np.arange(id_base, id_base + n_mine, dtype=np.int32)
    else:
        db = sw.Database(handle, res, offs, long_threshold=(args.long_threshold or None))
        sampler = host_sampler(res, offs)
        sampler.full = (res, offs)
        id_base = None
    n = len(offs) - 1
    residues = int(offs[-1])
    st = db.stats()
    log("rank %d: share %d/%d: %d subjects, %d residues, generated + packed + resident in %.1fs: %s"
        % (rank, shard_rank, shard_world, n, residues, time.perf_counter() - t0, st))

    # a ring of score buffers: the top-K exchange of step i (on its own
    # stream) overlaps the scans after it; with 8 buffers the exchange that
    # last read a buffer has finished long before the buffer is scanned into
    # again, so the scan's stream usually needs no wait packet for it
    NBUF = 8
    scores_buf = [torch.zeros((nq, max(n, 1)), dtype=torch.int32, device=dev) for _ in range(NBUF)]
    K = args.topk
    top = torch.empty((nq, K), dtype=torch.int64, device=dev)
    # rows of the gathered top-K: the ranks (or the rehearsed ranks)
    xworld = shard_world if args.rehearse_exchange else world
    gathered = torch.empty((xworld, nq, K), dtype=torch.int64, device=dev)
    final = torch.empty((nq, K), dtype=torch.int64, device=dev)
    gid_dev = torch.from_numpy(gids).to(dev) if id_base is None else None

    mat = sw.capi.builtin_matrix(MATRICES[args.matrix])
    scoring = (mat, args.gap_open, args.gap_extend)

    # The exchange (device top-K, RCCL all-gather, merge) runs on a second
    # stream with its own library handle, so it overlaps the next step's scan
    # (HIP events order the two; --no-overlap runs everything on one stream).
    xstream = stream if args.no_overlap else torch.cuda.Stream(dev, priority=args.exchange_priority)
    xhandle = handle
    if not args.no_overlap:
        xhandle = sw.Handle(gpu)
        xhandle.set_stream(xstream.cuda_stream)
    ranked = [torch.cuda.Event() for _ in range(NBUF)]
    counter = [0]

    def step():
        b = counter[0] % NBUF
        counter[0] += 1
        scores = scores_buf[b]
        # step i-NBUF's top-K has read this buffer (a wait is a packet the
        # command processor spends ~5 us on: skipped when the host already
        # sees the event complete)
        if counter[0] > NBUF and not ranked[b].query():
            stream.wait_event(ranked[b])
        if nq == 1:
            db.scan_device(queries[0], scores.data_ptr(), *scoring)
        else:
            db.scan_batch_device(queries, scores.data_ptr(), *scoring)
        # the exchange waits for the scan's own end event (no record here)
        if xstream is not stream:
            handle.stream_wait_scan(xstream.cuda_stream)
        with torch.cuda.stream(xstream):
            # device top-K per query: int64 keys (score << 32 | 2^31-1-global id), best first
            for k in range(nq):
                if gid_dev is not None:
                    xhandle.topk_device_ids(scores[k].data_ptr(), n, gid_dev.data_ptr(), K, top[k].data_ptr())
                else:
                    xhandle.topk_device(scores[k].data_ptr(), n, K, top[k].data_ptr(), id_base=id_base)
            if world > 1:
                if args.backend == "nccl":
                    tdist.all_gather_into_tensor(gathered, top)  # RCCL over xGMI: nq x K x 8 B per rank
                else:
                    parts = [torch.empty((nq, K), dtype=torch.int64) for _ in range(world)]
                    tdist.all_gather(parts, top.cpu())
                    gathered.copy_(torch.stack(parts))
            elif args.rehearse_exchange:
                tdist.all_gather_into_tensor(gathered[:1], top)
                gathered[1:].copy_(top.unsqueeze(0).expand(xworld - 1, nq, K))
            if xworld > 1:
                for k in range(nq):
                    merged = gathered[:, k, :].contiguous()
                    xhandle.topk_keys_device(merged.data_ptr(), xworld * K, K, final[k].data_ptr())
            ranked[b].record(xstream)

    cells_rank = float(qtot) * residues

    def one_step_ms():
        """One step alone, synchronised on both sides (host wall clock)."""
        torch.cuda.synchronize()
        t = time.perf_counter()
        step()
        torch.cuda.synchronize()
        return round((time.perf_counter() - t) * 1e3, 4)

    def timed_loop(steps=None, warmup=None):
        """W untimed steps, then K timed steps between barrier + sync pairs;
        returns (max-over-ranks seconds, all ranks' cells per step, kernel
        timing, name of the per-wave inter kernel)."""
        steps = args.steps if steps is None else steps
        for _ in range(args.warmup if warmup is None else warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            tdist.barrier()
        torch.cuda.synchronize()
        handle.timing_reset()
        t_start = time.perf_counter()
        for _ in range(steps):
            step()
        t_enq = time.perf_counter() - t_start  # host time to enqueue the K steps
        torch.cuda.synchronize()
        if world > 1:
            tdist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t_start
        log("rank %d: %d steps in %.3f ms, host enqueue %.3f ms" % (rank, steps, elapsed * 1e3, t_enq * 1e3))
        kt = handle.timing_total()
        if world > 1:
            t = torch.tensor([elapsed, cells_rank], dtype=torch.float64,
                             device=dev if args.backend == "nccl" else "cpu")
            tmax = t.clone()
            tdist.all_reduce(tmax, op=tdist.ReduceOp.MAX)
            tdist.all_reduce(t, op=tdist.ReduceOp.SUM)
            return float(tmax[0]), float(t[1]), kt, (handle.last_kernel(), handle.last_intra_kernel())
        return elapsed, cells_rank, kt, (handle.last_kernel(), handle.last_intra_kernel())

    # the first step on this database (and scoring): lazy allocations, the
    # merged launch's table, the adaptive routing's first observation
    cold_first = one_step_ms()
    elapsed_max, cells_all, kt, (kernel, intra_kernel) = timed_loop()
    st = db.stats()  # the coop split of the timed scans
    sustained = None
    if args.sustained_seconds > 0:
        # back to back for >= the stated seconds (every rank runs the same
        # count: from the timed region's max-over-ranks step time)
        n_sus = max(args.steps, int(math.ceil(args.sustained_seconds / (elapsed_max / args.steps))))
        s_elapsed, s_cells, s_kt, _ = timed_loop(steps=n_sus, warmup=0)
        sustained = sustained_summary(s_elapsed, n_sus, s_cells, s_kt["wave_ms"], s_kt["scans"], world)
    final_keys = (final if world > 1 else top).cpu().numpy()
    top_ids, top_scores = sw.capi.decode_keys(final_keys[0])
    # the measured run's scores and keys (its last step's buffer), for the parity leg
    gs = scores_buf[(counter[0] - 1) % NBUF].cpu().numpy()[:, :n]
    dev_top = top.cpu().numpy()
    # a cold scan next to a warm one: the adaptive routing (which kernel
    # forms a scan runs depends on what earlier scans of this database
    # observed: the int16 span of the widest blocks, the intra order) forgotten
    # by sw_db_reset_adaptive, then the same step again
    db.reset_adaptive()
    cold_warm = {"first_scan_ms": cold_first, "after_reset_adaptive_ms": one_step_ms(), "warm_ms": one_step_ms(),
                 "timed_ms_per_step": round(elapsed_max * 1e3 / args.steps, 4),
                 "note": "single steps synchronised on both sides (host clock, launch latency included): the "
                         "database's first step, one after sw_db_reset_adaptive, one after that"}

    ref = None
    r_parity = None
    if not args.no_reference_scoring:
        scoring = (sw.capi.builtin_matrix(0), 2, 2)  # SWSolver.cu:54-81, GAP_PENALTY 2 (:7)
        r_cold = one_step_ms()
        r_elapsed, r_cells, r_kt, r_kernel = timed_loop()
        # its last step's scores and keys, re-checked against the oracle below
        r_parity = (scores_buf[(counter[0] - 1) % NBUF].cpu().numpy()[:, :n], top.cpu().numpy(),
                    (final if world > 1 else top).cpu().numpy(), scoring)
        scoring = (mat, args.gap_open, args.gap_extend)

    eff, aff, quota = host_cores()
    # the parity leg runs on every rank at once: split this host's cores
    vthreads = max(1, (args.cpu_threads or eff) // max(1, local_world))
    verify_res, verify_ok = None, None
    if not args.no_verify:
        verify_res, verify_ok = verify(sw, sw.dist, world, rank, queries, sampler, n, gids, gs, dev_top, final_keys,
                                       K, scoring, vthreads, args.verify_seconds, args.backend)
    if r_parity is not None:
        r_res, r_ok = None, None
        if not args.no_verify:
            r_gs, r_top, r_final, r_scoring = r_parity
            r_res, r_ok = verify(sw, sw.dist, world, rank, queries, sampler, n, gids, r_gs, r_top, r_final, K,
                                 r_scoring, vthreads, args.verify_seconds, args.backend)
        ref = reference_scoring_summary(r_elapsed, r_cells, args.steps, r_kt, r_kernel, r_cold, r_res, r_ok)

    if rank == 0:
        value = cells_all * args.steps / elapsed_max / 1e9
        ms_step = elapsed_max * 1e3 / args.steps
        nsc = max(kt["scans"], 1)
        inter_ms = kt["inter_ms"] / nsc
        intra_ms = kt["intra_ms"] / nsc
        wave_ms = kt["wave_ms"] / nsc
        coop_ms = kt["coop_ms"] / nsc
        # Dominant kernel: the per-wave inter-sequence kernel (most of the
        # cells; the intra kernel takes the long subjects beside it on a side
        # stream; int32 paths also run a cooperative kernel on the widest
        # blocks).  Its duration is HIP events around its launch on its own
        # stream, per scan (per query for c3).  Algorithmic bytes per launch
        # (SURVEY.md §8d): 1 B per residue it scans + 12 B per subject
        # (offset, length, int32 score).
        lens_desc = np.sort(offs[1:] - offs[:-1])[::-1]
        n_inter = n - st["n_long"]
        inter_res = residues - int(lens_desc[:st["n_long"]].sum())
        # blocks of a separate cooperative / wave-pair launch are not the
        # dominant kernel's; merged pairs are part of it
        side_blocks = st["coop_blocks"] + (0 if st["pair_merged"] else st["pair_blocks"])
        side_res = st["coop_residues"] + (0 if st["pair_merged"] else st["pair_residues"])
        n_coop = min(side_blocks * 64, n_inter)
        wave_res = inter_res - side_res
        alg_bytes = wave_res + 12 * (n_inter - n_coop)
        kernel_ms = wave_ms
        wave_gcups = float(qtot) / nq * wave_res / (wave_ms * 1e-3) / 1e9 if wave_ms > 0 else 0.0
        intra_res = residues - inter_res
        roof_kernel = kernel
        if nq > 1 and "sw_inter_x2" in kernel and "+lpt" not in kernel:
            # a batch (C3): the queries' inter scans run different forms
            # (single waves for short queries, wave pairs for longer ones);
            # the roofline covers them all, per query
            roof_kernel = "sw_inter_x2* (per query of the batch)"
        if "+lpt" in kernel:
            # one merged launch (sw_scan_lpt) scans every subject: the inter
            # blocks and the long subjects' fp16 pass, longest work first
            wave_res = residues
            alg_bytes = residues + 12 * n
            wave_gcups = float(qtot) / nq * residues / (wave_ms * 1e-3) / 1e9 if wave_ms > 0 else 0.0
        elif intra_res > inter_res:
            # long-subject regime (C5): the intra kernel scans most cells
            roof_kernel = intra_kernel
            alg_bytes = intra_res + 12 * st["n_long"]
            kernel_ms = intra_ms
            wave_gcups = float(qtot) / nq * intra_res / (intra_ms * 1e-3) / 1e9 if intra_ms > 0 else 0.0
        achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
        traffic, traffic_note = None, "no rocprofv3 --pmc measurement of this workload and build"
        valu_hw = None
        affine = args.gap_open != args.gap_extend
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            tj = traffic_entry(tj, workload_key(args, qtot)) or {}
            if not args.shard_of and world == 1 and tj.get("kernel") == roof_kernel:
                if tj.get("kernel_src_sha16") == kernel_source_hash():
                    traffic = tj.get("hbm_bytes_per_launch")
                    if tj.get("sq_insts_valu_per_launch") and tj.get("profiled_ns_per_launch") and kernel_ms > 0:
                        # hardware-anchored VALU fraction of the dominant
                        # launch: its SQ_INSTS_VALU (wave instructions) at the
                        # measured packed-op cost, over every SIMD's cycles at
                        # the clock GRBM_GUI_ACTIVE shows under this load
                        insts = tj["sq_insts_valu_per_launch"]
                        # GRBM_GUI_ACTIVE is summed over the 8 XCDs by rocprofv3:
                        # /8 = the cycles of the profiled launch itself, so the
                        # fraction uses that one pass's clock AND duration
                        cyc = tj["grbm_gui_active_per_launch"] / 8
                        clk = cyc / tj["profiled_ns_per_launch"]  # GHz
                        intra_dom = roof_kernel == intra_kernel
                        cells_launch = float(qtot) / nq * (intra_res if intra_dom else wave_res)
                        per128 = insts / (cells_launch / 128)
                        valu_hw = {"sq_insts_valu_per_launch": insts,
                                   "valu_insts_per_128_cells": round(per128, 3),
                                   "clock_ghz_under_load": round(clk, 3),
                                   "profiled_ms_per_launch": round(tj["profiled_ns_per_launch"] * 1e-6, 4),
                                   "cycles_per_valu_inst": 4.25,
                                   "issue_frac": round(insts * 4.25 / (SIMDS * cyc), 4),
                                   "issue_frac_4cyc": round(insts * 4.0 / (SIMDS * cyc), 4),
                                   "source": "stored rocprofv3 --pmc SQ pass (pmc_traffic.json), same kernel sources; "
                                             "instructions, cycles and duration all of that one profiled launch"}
                        if intra_dom and "<" in roof_kernel:
                            # a wave-step of sw_intra_x2<RI> is 64 lanes x RI rows x 2 subjects
                            ri = int(roof_kernel.split("<")[1].split(">")[0].split(",")[0])
                            valu_hw["valu_insts_per_wave_step"] = round(per128 * ri, 1)
                        if tj.get("sq_lds_bank_conflict_per_launch") and tj.get("sq_active_inst_lds_per_launch"):
                            valu_hw["lds_bank_conflict_cycles_per_lds_inst"] = round(
                                tj["sq_lds_bank_conflict_per_launch"] / tj["sq_active_inst_lds_per_launch"], 3)
                    traffic_note = ("stored rocprofv3 --pmc measurement (FETCH_SIZE x2 + WRITE_SIZE) of this "
                                    "workload, taken on a build with the same kernel sources (%s, %s)"
                                    % (tj.get("kernel_src_sha16"), tj.get("measured", "?")))
                else:
                    traffic_note = "stored PMC measurement is of other kernel sources; not reported"
        except (OSError, ValueError):
            pass
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GCUPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": ("fp16" if ("fp16" in roof_kernel or "intra_x2" in roof_kernel)
                      else "int16" if "_x2" in roof_kernel else "int32"),
            "dtype_note": "the DP cells compute in packed 16-bit pairs (fp16 holds every integer in [-2048, "
                          "2048] exactly and the cells are offset by -2048 + 2 ge, so scores up to ~4,000 stay "
                          "exact; a lane whose maximum nears that bound is re-scored in int16, then int32); "
                          "scores are bit-exact int32",
            "data": "synthetic",
            "config": {
                "workload": "%s, %d subjects (%d on this rank's share, %d residues), %s, gap open %d / extend "
                            "%d%s, top-%d all-gathered" % (
                                desc, args.db_seqs, n, residues, args.matrix.upper(), args.gap_open,
                                args.gap_extend,
                                " (BLAST 11/1)" if (args.gap_open, args.gap_extend) == (12, 1) else "", K),
                "config": args.config,
                "scoring": {"matrix": args.matrix, "gap_open": args.gap_open, "gap_extend": args.gap_extend},
                "queries": qnames if nq > 1 else qnames[0], "query_residues": int(qtot),
                "database_subjects": args.db_seqs,
                "subjects_rank0": n, "residues_rank0": residues,
                "sharding": ("id range of the database per rank" if args.config == "c4" else
                             "LPT over subject lengths (residue-balanced) of one database"),
                "parallelism": "db-shard x%d + RCCL allgather top-K" % world,
                "long_threshold": st["long_threshold"], "long_subjects_rank0": st["n_long"],
                "cells_per_step": cells_all,
            },
            "kernel_ms_per_scan": {"inter_phase": round(inter_ms, 4), "sw_inter": round(wave_ms, 4),
                                   "sw_inter_coop": round(coop_ms, 4), "sw_intra": round(intra_ms, 4),
                                   "scan_total": round(kt["total_ms"] / nsc, 4)},
            "cells_split_per_step_rank0": {"sw_inter": float(qtot) * (inter_res - side_res),
                                           "sw_inter_coop": float(qtot) * side_res,
                                           "sw_intra": float(qtot) * (residues - inter_res)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": traffic, "traffic_note": traffic_note,
                         "kernel": roof_kernel, "workload_key": workload_key(args, qtot),
                         "alg_bytes_per_launch": int(alg_bytes), "kernel_ms": round(kernel_ms, 4)},
            "valu_roofline": valu_roofline(roof_kernel, cells_all / world, kt["total_ms"] / nsc * nq, wave_gcups,
                                           affine, (valu_hw or {}).get("clock_ghz_under_load")),
            "valu_hw": valu_hw,
            "cold_first_scan_ms": cold_first,
            "cold_warm": cold_warm,
            "kernels": {"inter": kernel, "intra": intra_kernel},
            # each step's device top-K: one launch per query (sw_topk.hip
            # sw_topk_fused) on the exchange stream, beside the next scan
            "topk": "one launch per query on the exchange stream, beside the next scan"
                    if not args.no_overlap else "after the scan, its stream",
            "top_hit": {"id": int(top_ids[0]), "score": int(top_scores[0])},
            "host": {"cores_used": args.cpu_threads or eff, "affinity_cpus": aff, "cgroup_quota_cpus": quota},
        }
        if args.shard_of:
            out["rehearsal"] = "rank %d's share of %d GPUs measured alone on one GPU" % (shard_rank, shard_world)
            if args.rehearse_exchange:
                out["exchange_rehearsed"] = ("each step: device top-%d, a one-rank RCCL all-gather, %d rows "
                                             "copied in, the device merge of %d x %d keys, on the exchange "
                                             "stream beside the next scan" % (K, shard_world - 1, shard_world, K))
        if ref is not None:
            out["reference_scoring"] = ref
        if sustained is not None:
            out["sustained"] = sustained
        if verify_res is not None:
            out["parity"] = verify_res
            out["parity_sample_ok"] = verify_ok
            if ref is not None and ref.get("parity_ok") is not None:
                # every scoring the line reports is checked
                out["parity_sample_ok"] = bool(verify_ok and ref["parity_ok"])
        if not args.no_cpu_baseline and world == 1 and not args.shard_of:
            threads = args.cpu_threads or eff
            cb, cparity = cpu_baseline(queries, sampler, n, gs, args.cpu_seconds, threads, scoring,
                                       args.cpu_seconds / 2)
            out["cpu_baseline"] = cb
            out["parity_sample_ok"] = bool(cparity and out.get("parity_sample_ok", True))
        print(json.dumps(out), flush=True)
    if world > 1:
        tdist.barrier()
    if tdist.is_initialized():
        tdist.destroy_process_group()
    db.close()
    if xhandle is not handle:
        xhandle.close()
    handle.close()


if __name__ == "__main__":
    main()
