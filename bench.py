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
50,000,000-subject database split over the ranks (configs[3]; strong
scaling), each rank's shard generated in its GPU's HBM from (seed, global
id) by the counter-based generator (sw_db_create_synthetic); --config c5: a
5,000-residue synthetic query against 10,000 subjects of N(2000, 200)
residues (configs[4]).  These are the other BASELINE configurations,
measured with the same code; the driver's headline is the default (c2).

One step = one pass of the hot path over the rank's resident shard: build the
query profile(s), run the scan kernels (intra-sequence for subjects longer
than the long threshold, inter-sequence for the rest), then the top-K
exchange (device top-K per query, RCCL all-gather of K (score, id) keys per
rank, device merge).

Multi-GPU (torchrun, one process per GPU): every rank holds its OWN shard of
the same size (weak scaling; shard = the rank's seed), so the global database
grows with N (config C4's pattern).  value = all cells processed by all ranks
/ the max-over-ranks time of K steps.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
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
    # the same cells with the widest blocks run by wave pairs in the same launch
    "sw_inter_x2p<32,8,affine,fp16>": (5.91 * 4.25 + 0.305 * 2.7) / 128,
    "sw_inter_x2p<32,8,linear>": (5.0 * 4.25 + 0.29 * 2.7) / 128,
    # per 2 x 64 cells: 4.53 v_pk_max_i16, 2.65 v_pk_sub_u16, 0.94 v_pk_mad_u16
    "sw_inter_x2p<32,8,affine>": (8.117 * 4.25) / 128,
    "sw_inter_x2s<32,8,affine>": (8.117 * 4.25) / 128,
    "sw_inter_x2s<48,4,linear>": (4.688 * 4.25) / 128,
    "sw_inter_x2<32,8,affine>": ((4.83 + 2.83 + 1) * 4.25 + 2.7) / 128,
    "sw_inter_x2<16,16,affine>": ((4.87 + 2.87 + 1) * 4.25 + 2.7) / 128,
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
# lane-63 collection; hipcc -S of sw_intra_x2.hip)
for _ri in (4, 8, 12, 16):
    VALU_MODEL["sw_intra_x2<%d>" % _ri] = (_ri * (6.78 * 4.25) + 80.0) / (128 * _ri)
MATRICES = {"blosum50": 0, "blosum62": 1}
SEED = 1782
C4_TOTAL = 50_000_000
C3_QUERIES = ["P02232", "P05013", "P14942", "P07327", "P01008", "P03435", "P42357", "P21177",
              "Q38941", "P27895", "P07756", "P04775", "P19096", "P28167", "P0C6B8", "P20930",
              "P08519", "Q7TMA5", "P33450", "Q9UKN1"]


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def read_query(name):
    with open(os.path.join(REPO, "tests", "golden", "queries", name + ".fasta")) as f:
        return "".join(f.read().split("\n")[1:])


def workload_key(args, qlen):
    return "%s/%d/%d/%s-%d-%d" % (args.query, args.db_seqs, qlen, args.matrix, args.gap_open, args.gap_extend)


def valu_roofline(kernel, cells_rank, scan_ms, kernel_gcups):
    """The binding roofline: VALU instruction issue.  peak = the modeled
    issue-bound rate of the per-wave inter kernel (VALU_MODEL), achieved =
    the whole scan's rate (all kernels of the scan, concurrent)."""
    cpc = VALU_MODEL.get(kernel.split("+")[0])  # "+int16[0,n)": the widest blocks in int16 beside it
    if cpc is None or scan_ms <= 0:
        return None
    peak = SIMDS * CLOCK_HZ / cpc / 1e9
    achieved = cells_rank / (scan_ms * 1e-3) / 1e9
    return {"bound": "valu-issue", "achieved": round(achieved, 1), "peak": round(peak, 1), "unit": "GCUPS",
            "frac": round(achieved / peak, 4), "kernel": kernel, "simd_cycles_per_cell": round(cpc, 5),
            "kernel_alone_gcups_while_concurrent": round(kernel_gcups, 1)}


def host_sampler(res, offs):
    """Subjects idx of a host-generated shard as (residues, offsets)."""
    def take(idx):
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


def cpu_baseline(sw, queries, sampler, n, gpu_scores, seconds, threads, scoring):
    """The oracle (C restatement of cpu.cpp's recurrence, Gotoh for affine;
    kind "port") on a bounded random sample of the same shard, every query of
    the workload, on this host's cores, with the same scoring as the GPU run.
    sampler(idx) -> (residues, offsets) of shard subjects idx; gpu_scores:
    [nq][n] scores of the measured run (parity check)."""
    mat, go, ge = scoring
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import sw_oracle
    rng = np.random.default_rng(1782)
    perm = rng.permutation(n)

    def sample(m):
        idx = np.sort(perm[:m])
        sr, so = sampler(idx)
        return idx, sr, so

    def run(sr, so):
        return [sw_oracle.scan(q, sr, so, mat=mat, gap_open=go, gap_extend=ge, nthreads=threads) for q in queries]

    # calibrate on growing samples until one takes >= 0.5 s (thread start-up
    # dominates tiny samples), then size the real one to ~`seconds`
    m0 = min(n, 200)
    while True:
        idx, sr, so = sample(m0)
        t = time.perf_counter()
        run(sr, so)
        dt = max(time.perf_counter() - t, 1e-3)
        if dt >= 0.5 or m0 >= n:
            break
        m0 = min(n, m0 * 4)
    m = int(min(n, max(m0, m0 * seconds / dt)))
    idx, sr, so = sample(m)
    t = time.perf_counter()
    cpu = run(sr, so)
    dt = time.perf_counter() - t
    qtot = sum(len(q) for q in queries)
    cells = qtot * int(so[-1])
    parity = all(bool(np.array_equal(c, gpu_scores[k][idx])) for k, c in enumerate(cpu))
    return {"value": round(cells / dt / 1e9, 4), "unit": "GCUPS", "cores": threads, "kind": "port",
            "sample": "%d of %d subjects (%d residues) of rank 0's shard x %d quer%s (%d residues), %.3g cells, "
                      "%.1f s on %d threads; scores equal to the GPU's: %s"
                      % (m, n, int(so[-1]), len(queries), "y" if len(queries) == 1 else "ies", qtot, cells, dt,
                         threads, parity)}, parity


def make_workload(sw, args, rank):
    """(queries [code arrays], query names, residues, offsets, description)."""
    if args.config == "c2":
        res, offs = sw.synth.database(args.db_seqs, shard=rank)
        return [sw.encode(read_query(args.query))], [args.query], res, offs, \
            "C2: query %s (%d aa) vs synthetic Swiss-Prot-sized db" % (args.query, len(read_query(args.query)))
    if args.config == "c4":
        return [sw.encode(read_query(args.query))], [args.query], None, None, \
            "C4: query %s (%d aa) vs a %d-subject synthetic db generated on the devices" % (
                args.query, len(read_query(args.query)), C4_TOTAL)
    if args.config == "c3":
        res, offs = sw.synth.database(args.db_seqs, shard=rank)
        qs = [sw.encode(read_query(n)) for n in C3_QUERIES]
        return qs, C3_QUERIES, res, offs, \
            "C3: batch of the %d shipped queries (%d..%d aa, sum %d) vs synthetic Swiss-Prot-sized db" % (
                len(qs), min(map(len, qs)), max(map(len, qs)), sum(map(len, qs)))
    # c5: one 5,000-residue query vs 10,000 subjects of N(2000, 200)
    res, offs = sw.synth.fixed_length_database(args.db_seqs, 2000, 200, shard=rank)
    return [sw.synth.query(5000)], ["synthetic-5000"], res, offs, \
        "C5: synthetic 5000-aa query vs N(2000, 200)-residue subjects"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5"],
                    help="c2 = the headline (BASELINE configs[1]); c3 / c4 / c5 = configs[2] / [3] / [4]")
    ap.add_argument("--steps", type=int, default=None, help="default 10 (c2, c5) / 3 (c3)")
    ap.add_argument("--warmup", type=int, default=None, help="default 2 (c2, c5) / 1 (c3)")
    ap.add_argument("--db-seqs", type=int, default=None,
                    help="subjects per rank (default 570000; c4: 50M / ranks; c5: 10000)")
    ap.add_argument("--query", default="P07327")
    ap.add_argument("--topk", type=int, default=100)
    ap.add_argument("--matrix", default="blosum62", choices=sorted(MATRICES))
    ap.add_argument("--gap-open", type=int, default=12, help="cost of a 1-residue gap (BLAST 11/1 -> 12)")
    ap.add_argument("--gap-extend", type=int, default=1)
    ap.add_argument("--no-reference-scoring", action="store_true",
                    help="skip the second timed loop with the reference's BLOSUM50 / linear 2")
    ap.add_argument("--long-threshold", type=int, default=0, help="0 = library default")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # the latest rocprofv3 --pmc measurement of the C2 launch (FETCH_SIZE x2 +
    # WRITE_SIZE, scripts/pmc_traffic.py); kept at the root because profiles/
    # does not travel to the GPU box
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "pmc_traffic.json"))
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo = rehearse the multi-rank path on one GPU (CPU collectives)")
    ap.add_argument("--device", type=int, default=None, help="override the GPU index (rehearsal)")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = 3 if args.config == "c3" else 10
    if args.warmup is None:
        args.warmup = 1 if args.config == "c3" else 2
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.db_seqs is None:
        args.db_seqs = {"c5": 10000, "c4": -(-C4_TOTAL // world_env)}.get(args.config, 570000)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    gpu = local if args.device is None else args.device
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)

    import _swpkg
    sw = _swpkg.load()

    t0 = time.perf_counter()
    queries, qnames, res, offs, desc = make_workload(sw, args, rank)
    nq = len(queries)
    qtot = sum(len(q) for q in queries)

    handle = sw.Handle(gpu)
    # The library launches on a torch stream (not the legacy null stream,
    # whose handle is 0 = "library-owned stream" for sw_set_stream), so the
    # scan is stream-ordered with the top-K ops that read its scores.
    stream = torch.cuda.Stream(dev)
    handle.set_stream(stream.cuda_stream)
    torch.cuda.set_stream(stream)
    if res is None:  # c4: the shard is generated in this GPU's HBM
        id_base = rank * args.db_seqs
        db = sw.Database.synthetic(handle, SEED, args.db_seqs, id_base=id_base,
                                   long_threshold=(args.long_threshold or None))
        lens, _ = db.subjects()
        offs = np.zeros(len(lens) + 1, dtype=np.int64)
        offs[1:] = np.cumsum(lens)
        sampler = counter_sampler(sw, SEED, id_base)
    else:
        db = sw.Database(handle, res, offs, long_threshold=(args.long_threshold or None))
        sampler = host_sampler(res, offs)
    n = len(offs) - 1
    residues = int(offs[-1])
    st = db.stats()
    log("rank %d: shard %d subjects, %d residues, generated + packed + resident in %.1fs: %s"
        % (rank, n, residues, time.perf_counter() - t0, st))

    scores = torch.zeros((nq, n), dtype=torch.int32, device=dev)
    K = min(args.topk, n)
    top = torch.empty((nq, K), dtype=torch.int64, device=dev)
    gathered = torch.empty((world, nq, K), dtype=torch.int64, device=dev)
    final = torch.empty((nq, K), dtype=torch.int64, device=dev)

    mat = sw.capi.builtin_matrix(MATRICES[args.matrix])
    scoring = (mat, args.gap_open, args.gap_extend)

    def step():
        if nq == 1:
            db.scan_device(queries[0], scores.data_ptr(), *scoring)
        else:
            db.scan_batch_device(queries, scores.data_ptr(), *scoring)
        # device top-K per query: int64 keys (score << 32 | 2^31-1-global id), best first
        for k in range(nq):
            handle.topk_device(scores[k].data_ptr(), n, K, top[k].data_ptr(), id_base=rank * n)
        if world == 1:
            return
        if args.backend == "nccl":
            dist.all_gather_into_tensor(gathered, top)  # RCCL over xGMI: nq x K x 8 B per rank
        else:
            parts = [torch.empty((nq, K), dtype=torch.int64) for _ in range(world)]
            dist.all_gather(parts, top.cpu())
            gathered.copy_(torch.stack(parts))
        for k in range(nq):
            merged = gathered[:, k, :].contiguous()
            handle.topk_keys_device(merged.data_ptr(), world * K, K, final[k].data_ptr())

    cells_rank = float(qtot) * residues

    def timed_loop():
        """W untimed steps, then K timed steps between barrier + sync pairs;
        returns (max-over-ranks seconds, all ranks' cells per step, kernel
        timing, name of the per-wave inter kernel)."""
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        handle.timing_reset()
        t_start = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t_start
        kt = handle.timing_total()
        if world > 1:
            t = torch.tensor([elapsed, cells_rank], dtype=torch.float64,
                             device=dev if args.backend == "nccl" else "cpu")
            tmax = t.clone()
            dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            return float(tmax[0]), float(t[1]), kt, (handle.last_kernel(), handle.last_intra_kernel())
        return elapsed, cells_rank, kt, (handle.last_kernel(), handle.last_intra_kernel())

    elapsed_max, cells_all, kt, (kernel, intra_kernel) = timed_loop()
    st = db.stats()  # the coop split of the timed scans
    final_keys = (final if world > 1 else top).cpu().numpy()
    top_ids, top_scores = sw.capi.decode_keys(final_keys[0])
    gs = scores.cpu().numpy() if (not args.no_cpu_baseline and world == 1 and rank == 0) else None

    ref = None
    if not args.no_reference_scoring:
        scoring = (sw.capi.builtin_matrix(0), 2, 2)  # SWSolver.cu:54-81, GAP_PENALTY 2 (:7)
        r_elapsed, r_cells, r_kt, r_kernel = timed_loop()
        r_n = max(r_kt["scans"], 1)
        ref = {"scoring": "BLOSUM50 (SWSolver.cu:54-81), linear gap 2 (the reference's own)",
               "value": round(r_cells * args.steps / r_elapsed / 1e9, 2), "unit": "GCUPS",
               "ms_per_step": round(r_elapsed * 1e3 / args.steps, 3), "kernel": r_kernel[0],
               "intra_kernel": r_kernel[1],
               "kernel_ms_per_scan": {"sw_inter": round(r_kt["wave_ms"] / r_n, 4),
                                      "sw_inter_coop": round(r_kt["coop_ms"] / r_n, 4),
                                      "sw_intra": round(r_kt["intra_ms"] / r_n, 4),
                                      "scan_total": round(r_kt["total_ms"] / r_n, 4)}}

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
        if intra_res > inter_res:
            # long-subject regime (C5): the intra kernel scans most cells
            roof_kernel = intra_kernel
            alg_bytes = intra_res + 12 * st["n_long"]
            kernel_ms = intra_ms
            wave_gcups = float(qtot) / nq * intra_res / (intra_ms * 1e-3) / 1e9 if intra_ms > 0 else 0.0
        achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
        traffic = None
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if (args.config == "c2" and tj.get("workload_key") == workload_key(args, qtot)
                    and tj.get("kernel") == roof_kernel):
                traffic = tj.get("hbm_bytes_per_launch")
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
            "scaling": "strong" if args.config == "c4" else "weak",
            "vs_baseline": None,
            "dtype": ("fp16" if ("fp16" in roof_kernel or "intra_x2" in roof_kernel)
                      else "int16" if "_x2" in roof_kernel else "int32"),
            "dtype_note": "the DP cells compute in packed 16-bit pairs (fp16 holds every integer up to 2048 "
                          "exactly; a lane whose maximum nears that bound is re-scored in int16, then int32); "
                          "scores are bit-exact int32",
            "data": "synthetic",
            "config": {
                "workload": "%s, %d subjects/rank (%d residues/rank), %s, gap open %d / extend %d%s, top-%d "
                            "all-gathered" % (desc, n, residues, args.matrix.upper(), args.gap_open,
                                              args.gap_extend,
                                              " (BLAST 11/1)" if (args.gap_open, args.gap_extend) == (12, 1) else "",
                                              K),
                "config": args.config,
                "scoring": {"matrix": args.matrix, "gap_open": args.gap_open, "gap_extend": args.gap_extend},
                "queries": qnames if nq > 1 else qnames[0], "query_residues": int(qtot),
                "subjects_per_rank": n, "residues_per_rank": residues,
                "parallelism": "db-shard x%d + RCCL allgather top-K" % world,
                "long_threshold": st["long_threshold"], "long_subjects": st["n_long"],
                "cells_per_step": cells_all,
            },
            "kernel_ms_per_scan": {"inter_phase": round(inter_ms, 4), "sw_inter": round(wave_ms, 4),
                                   "sw_inter_coop": round(coop_ms, 4), "sw_intra": round(intra_ms, 4),
                                   "scan_total": round(kt["total_ms"] / nsc, 4)},
            "cells_split_per_step": {"sw_inter": float(qtot) * wave_res,
                                     "sw_inter_coop": float(qtot) * side_res,
                                     "sw_intra": float(qtot) * (residues - inter_res)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": traffic,
                         "kernel": roof_kernel,
                         "alg_bytes_per_launch": int(alg_bytes), "kernel_ms": round(kernel_ms, 4)},
            "valu_roofline": valu_roofline(roof_kernel, cells_all / world, kt["total_ms"] / nsc * nq, wave_gcups),
            "kernels": {"inter": kernel, "intra": intra_kernel},
            "top_hit": {"id": int(top_ids[0]), "score": int(top_scores[0])},
        }
        if ref is not None:
            out["reference_scoring"] = ref
        if gs is not None:
            threads = min(args.cpu_threads, os.cpu_count() or 1)
            cb, parity = cpu_baseline(sw, queries, sampler, n, gs, args.cpu_seconds, threads,
                                      scoring=(mat, args.gap_open, args.gap_extend))
            out["cpu_baseline"] = cb
            out["parity_sample_ok"] = parity
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    db.close()
    handle.close()


if __name__ == "__main__":
    main()
