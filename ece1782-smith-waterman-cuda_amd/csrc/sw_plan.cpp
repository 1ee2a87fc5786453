// sw_plan.cpp — the host driver's scan-planning policies (SURVEY.md §8 row
// a2; the reference packs one fixed 32-lane block order per launch,
// SWSolver.cu:309-359): which subjects go to the wavefront kernel, which
// blocks run by wave pairs, quads, 3-wave groups or tail pairs, and the
// longest-first work table of the merged launch (sw_scan_lpt) with its
// duration estimates.  Plain host code over a read-only view of a database
// (PlanDb); sw_capi.cpp owns the databases, caches the tables and uploads
// them.
#include "sw_plan.h"

#include <algorithm>
#include <cmath>
#include <utility>
#include <vector>

#include "sw_kernels.h"

namespace swplan {

// Subjects longer than this go to the wavefront kernel.  A 64-lane block of
// the inter kernel takes time proportional to its longest subject, so very
// long subjects would become the kernel's critical path; measured on the C2
// workload (mean length 360): 1536 beats 3072 by 1.3x and 1024 by 1.03x
// (profiles/r01_tune_inter.jsonl); with the cooperative kernel for wide
// blocks the best is ~2048 (profiles/r01_tune_coop.jsonl).  Default: 5.7 x
// mean length, clamped.

//
// Small databases: the inter kernels put one 64-subject block on a wave and
// need ~2 waves per SIMD (2048 blocks, ~131k subjects) to fill the chip.
// Below ~1000 blocks the one-wave-per-subject wavefront kernel is the faster
// path for subjects of a few hundred residues and up (config C5, 10,000
// subjects of ~2000 aa vs a 5000-aa query: 2.7 TCUPS all-intra vs 0.62 TCUPS
// inter, profiles/r01_c5/), so everything longer than 64 residues goes there.
constexpr int64_t kSmallDbSubjects = 64 * 1000;

// Databases smaller than ~kFillSubjects (C2's 570,000 subjects are ~4.3
// 64-subject blocks per wave slot of the 256-CU GPU) — e.g. a rank's share
// of a strong-scaled database — have too few blocks to hide the widest ones:
// the scan time becomes the widest block's latency (width x passes / 2 for
// a wave pair) while a long subject on the wavefront kernel takes only
// (length + 64) steps.  The threshold then shrinks as (n / kFillSubjects)^0.4,
// measured on C2's 1/2, 1/4 and 1/8 shares with the merged longest-first
// launch (profiles/r02_strong/: 1/8 best near 900; two concurrent launches
// preferred 1,536-2,048 / 1,024 / 600-704).
constexpr double kFillSubjects = 570000.0;

int32_t default_long_threshold(const PlanDb& db) {
    if (db.n == 0) return 1536;
    const double mean = static_cast<double>(db.residues) / static_cast<double>(db.n);
    if (db.n < kSmallDbSubjects && mean >= 256) return 64;
    const double fill = db.n < kSmallDbSubjects ? 1.0 : std::min(1.0, static_cast<double>(db.n) / kFillSubjects);
    const double t = 5.7 * mean * std::pow(fill, 0.4);
    return static_cast<int32_t>(std::min(8192.0, std::max(fill < 1.0 ? 512.0 : 1024.0, t)));
}

// Leading (widest) blocks handled by the cooperative kernel: blocks whose
// one-wave time is a large share of the whole scan.  One wave of a W-column
// block costs ~W*qpad*3.5 VALU instructions at ~8.4 cycles each (2 waves per
// SIMD); the scan costs ~16 cycles per 64 cells over 1024 SIMDs.  Measured on
// C2 (2.05e8 residues, profiles/r01_tune_coop.jsonl): width 384 with long
// threshold 2048 is best, i.e. W ~ sum(residues) / 530000.  sw_opts
// coop_width overrides (tuning); 0 disables.
int32_t coop_blocks(const PlanDb& db, int divisor) {
    // divisor from the inter kernel's shape (swk::inter_coop_divisor): the
    // two-subjects-per-lane kernel wants a wider cut-off than int32 (measured
    // on C2: 1024 beats 386 and 640, profiles/r01_x2/); 0 = no coop kernel
    const int32_t forced = db.opts->coop_width;
    if (divisor <= 0 && forced < 0) return 0;
    int64_t wmin = divisor > 0 ? std::max<int64_t>(128, db.residues / divisor) : 0;
    if (forced >= 0) wmin = forced;
    if (wmin <= 0) return 0;
    int32_t n = 0;
    while (n < static_cast<int32_t>(db.nblocks) &&
           static_cast<int64_t>(db.blk_groups[n]) * swk::kGroupCols >= wmin)
        ++n;
    return n;
}

// Leading (widest) blocks of a two-strips scan handled by wave pairs
// (sw_inter_x2p): blocks at least `width` columns wide, width =
// residues / kPairDivisor (1024 on C2: with the biased cell 1,024 beat 256,
// 512 and none by 2-4 %, profiles/r01_tail2/; sw_opts pair_width
// overrides; 0 disables).
constexpr int64_t kPairDivisor = 200000;

// Waves per group for those blocks: pairs; sw_opts pair_group = 4 runs quads.
// Measured on C2's 1/8 share (profiles/r02_strong/): the inter kernel alone
// is fastest with quads over every block >= 64 wide (1.08 ms vs 1.29 for
// pairs), but beside the concurrent long-subject kernel, whose workgroups
// are dispatched first, a quad waits for a whole free workgroup slot and the
// scan is slower (2.21 vs 1.77 ms).
int pair_group(const PlanDb& db) { return db.opts->pair_group == 4 ? 4 : 2; }

int32_t pair_blocks(const PlanDb& db) {
    int64_t wmin = std::max<int64_t>(256, db.residues / kPairDivisor);
    if (db.opts->pair_width >= 0) wmin = db.opts->pair_width;
    if (wmin <= 0) return 0;
    int32_t n = 0;
    while (n < static_cast<int32_t>(db.nblocks) &&
           static_cast<int64_t>(db.blk_groups[n]) * swk::kGroupCols >= wmin)
        ++n;
    return n;
}

// ---- one merged launch, longest work first (sw_scan_lpt) -----------------
// Estimated duration of each workgroup of the merged grid: an inter tick (8
// columns x 64 rows of a 64-subject block, one wave) ~7.4 us and an intra
// step of sw_intra_x2<RI> ~0.157 us at RI = 6, scaled by its modeled
// SIMD cycles (RI x 28.8 + 80) — measured on C2's 1/8 share
// (profiles/r02_strong/traces/).  Only the order matters: the dispatcher
// starts workgroups in grid order, so the longest work starts first.
constexpr double kTickUs = 7.4;
// (0.157 us alone on a SIMD; inside the busy merged grid a step takes ~0.3
// us, profiles/r04_*/: with the doubled cost the long subjects start early
// enough, C2's 1/8 share +0.8 %)
double intra_step_us(int ri) { return 2 * 0.157 * (ri * 28.8 + 80.0) / (6 * 28.8 + 80.0); }
// Under linear gaps the intra step is relatively dearer than under affine
// ones (C2's 1/8 share, profiles/r05_trace/: intra / inter item medians 0.31
// against 0.28); scaling its estimates for linear scans by 85, 120 or 140 %
// made the share's reference-scoring rate 1.8, 0.8 and 3.6 % lower
// (profiles/r05_ab/lpt_lin_intra/): the same cost as under affine gaps.

// The widest group blocks of the merged launch run by quads: those at least
// kQuadFrac x the long threshold wide, whose pair latency would otherwise
// exceed the long subjects' (sw_opts quad_width w: at least w columns; 0: none)
// — on databases of fewer than kQuadMaxFill x kFillSubjects subjects only.
// Measured (profiles/r04_sweep_quads/): without quads C2 +1.0 %, its 1/2
// share +2.5 %, 1/4 +1.8 %, C3 unchanged, but the 1/8 share -19.6 % (its
// widest blocks' pair latency sets the span there).
constexpr double kQuadFrac = 0.67;
constexpr double kQuadMaxFill = 0.2;

int32_t lpt_quad_blocks(const PlanDb& db, int32_t npair) {
    int64_t wmin = static_cast<int64_t>(kQuadFrac * db.long_threshold);
    if (static_cast<double>(db.n) >= kQuadMaxFill * kFillSubjects) wmin = 0;
    if (db.opts->quad_width >= 0) wmin = db.opts->quad_width;
    if (wmin <= 0) return 0;
    int32_t n = 0;
    while (n < npair && static_cast<int64_t>(db.blk_groups[n]) * swk::kGroupCols >= wmin) ++n;
    return n;
}

// ... or, under affine gaps, by 3-wave groups (InterArgs::blk_tri): a query
// of P passes takes ceil(P / 3) rounds instead of ceil(P / 4), no wave idle
// in the last round, and the workgroup's fourth wave runs a single-wave
// block (the widest singles, beside the widest groups) — used where the
// rounds are as few as the quads' (P = 1, 2, 3, 5, 6, 9: a 375-aa query is 6
// passes of 64 rows), for the group blocks at least kTriFrac x the long
// threshold wide (sw_opts tri_width w: at least w columns; 0: none), on the
// databases that run quads.  Measured on C2's shares (profiles/r06_tri/):
// the 1/8 share's slowest rank 8,551 -> 9,001 GCUPS at 430 of its 891 (the
// widest pair blocks, the launch's critical path, take two rounds of a tri
// instead of three of a pair: -32 % latency at the same wave time, the
// spare wave doing work a single-wave workgroup would); 350-460 all +3 to +5
// %; the 1/4 share +0.7 % at 700 (-0.3 % at 530), the 1/2 share -0.4 % at
// 1,300 and worse below, C2 -1.3 % at 1,500 and worse below.
constexpr double kTriFrac = 0.48;

int32_t lpt_tri_blocks(const PlanDb& db, int32_t npair, int passes) {
    int64_t wmin = static_cast<double>(db.n) < kQuadMaxFill * kFillSubjects
                       ? static_cast<int64_t>(kTriFrac * db.long_threshold) : 0;
    if (db.opts->tri_width >= 0) wmin = db.opts->tri_width;
    if (wmin <= 0 || passes <= 0 || (passes + 2) / 3 > (passes + 3) / 4) return 0;
    int32_t n = 0;
    while (n < npair && static_cast<int64_t>(db.blk_groups[n]) * swk::kGroupCols >= wmin) ++n;
    return n;
}

// The narrowest blocks of the merged launch run by wave pairs (x2p_wg's tail
// range): the launch's last-dispatched work is its narrowest single-wave
// workgroups, which start together once the rest is placed, and the longest
// of them sets the end — C2's last 10 % ran at 73 % of the workgroup slots,
// 4 % of the launch idle (profiles/r05_trace/).  Pairs halve those blocks'
// latency for a few % more wave time on them.  Default: half a round of
// pair workgroups (2 blocks each; 2 workgroups per CU: as many blocks as
// workgroup slots) when the single-wave workgroups fill the GPU more than
// twice over, a quarter of that for more single-wave blocks than slots;
// sw_opts tail_pairs n: the narrowest n blocks.  C2 (256 CUs) over
// 128-3,072 blocks: 512 best, +1.5 % (1,024 +0.8 %, 3,072 -0.4 %); its 1/4
// share with 128: +0.6 % affine, +0.9 % linear, its 1/2 share +2.4 %
// linear; the 1/8 share (432 single-wave blocks: none) -0.6 % with 128
// (profiles/r05_ab/tail_pairs/).
int32_t lpt_tail_blocks(const PlanDb& db, int32_t npair, int passes) {
    const int64_t singles = db.nblocks - npair;
    if (passes < 2 || singles < 2) return 0;
    int64_t n = 0;
    if (db.opts->tail_pairs >= 0) {
        n = db.opts->tail_pairs;
    } else {
        const int64_t slots = 2 * static_cast<int64_t>(db.cus);  // workgroups per CU: 2
        if (slots > 0 && singles > 2 * swk::kWavesPerWG * slots) n = slots;
        else if (slots > 0 && singles > slots) n = slots / 4;  // (C2's 1/2 and 1/4 shares)
    }
    return static_cast<int32_t>(std::min<int64_t>(n, singles - 1));
}

// Ticks of a single-wave block (x2s_block: chained passes when ncols >= 32).
double single_ticks(int64_t ncols, int passes) {
    if (ncols <= 0) return 0;
    if (ncols >= 32 && passes > 1) return static_cast<double>(passes) * ncols / 8 + 1;
    return static_cast<double>(passes) * (ncols / 8 + 1);
}

double group_ticks_host(int64_t ncols, int passes, int G) {
    if (ncols <= 0 || passes <= 0) return 0;
    const int64_t S = ncols / 8 + 1;
    const int64_t per = std::max<int64_t>(S, 3 * G);
    int64_t t = 0;
    for (int p = std::max(0, passes - G); p < passes; ++p) t = std::max<int64_t>(t, (p / G) * per + 3 * (p % G) + S);
    return static_cast<double>(t);
}


LptPlan lpt_plan(const PlanDb& db, int32_t qpad, int rows, int32_t qpad_intra, int ri, int32_t npair, int32_t nquad,
                 int32_t ntail, bool affine, bool tri) {
    const int passes = qpad / rows;
    const double tick_us = kTickUs * rows / 64;  // a tick: 8 columns of one pass
    const int64_t nb = db.nblocks;
    const int64_t pwg = nquad + (npair - nquad + 1) / 2;
    // blocks [tail, nb) by pairs (x2p_wg's clamp: none unless tail lies in (npair, nb))
    const int64_t tail = ntail > 0 && nb - ntail > npair && nb - ntail < nb ? nb - ntail : nb;
    // tris: the spare wave of tri workgroup g runs single block npair + g
    const int64_t nspare = tri ? std::max<int64_t>(0, std::min<int64_t>(nquad, tail - npair)) : 0;
    const int64_t s0 = npair + nspare;  // the single-wave workgroups' first block
    const int64_t swg = (tail - s0 + swk::kWavesPerWG - 1) / swk::kWavesPerWG;
    const int64_t twg = (nb - tail + 1) / 2;
    const int64_t npairs = (db.nlong + 1) / 2;
    const int64_t iwg = (npairs + swk::kWavesPerWG - 1) / swk::kWavesPerWG;
    const int nch = qpad_intra / (swk::kLanes * ri);
    const double step_us = intra_step_us(ri);
    std::vector<std::pair<double, int32_t>> w;
    w.reserve(static_cast<size_t>(pwg + swg + twg + iwg));
    auto width = [&](int64_t b) { return static_cast<int64_t>(db.blk_groups[b]) * swk::kGroupCols; };
    for (int64_t g = 0; g < nquad; ++g) {
        double c = group_ticks_host(width(g), passes, tri ? 3 : 4);
        if (g < nspare) c = std::max(c, single_ticks(width(npair + g), passes));
        w.emplace_back(c * tick_us, g);
    }
    for (int64_t g = nquad; g < pwg; ++g) {
        double c = 0;
        for (int q = 0; q < 2; ++q) {
            const int64_t b = nquad + (g - nquad) * 2 + q;
            if (b < npair) c = std::max(c, group_ticks_host(width(b), passes, 2));
        }
        w.emplace_back(c * tick_us, static_cast<int32_t>(g));
    }
    for (int64_t g = 0; g < swg; ++g)  // widest first: the workgroup's first block bounds it
        w.emplace_back(single_ticks(width(s0 + g * swk::kWavesPerWG), passes) * tick_us,
                       static_cast<int32_t>(pwg + g));
    for (int64_t g = 0; g < twg; ++g) {  // tail pairs: the first block of two is the wider
        w.emplace_back(group_ticks_host(width(tail + 2 * g), passes, 2) * tick_us,
                       static_cast<int32_t>(pwg + swg + g));
    }
    // The longest pairs whose one-wave latency would exceed every inter
    // item's run in the pipelined form (a 128-row query chunk per wave,
    // ix2::intra_x2_wg PIPE; at most 4 chunks): a pair of one outlier subject
    // otherwise sets the launch's span alone (C2's 1/8 share: the 7,429-aa
    // subject's workgroup 1,275 us, every other one <= 1,224 us; pipelined,
    // 7,662 -> 8,082 GCUPS on one box, profiles/r04_*/).  They start first.
    // SW_LPT_PIPE=n forces n pairs (tests).
    const int nchp = (qpad_intra + 127) / 128;
    double inter_max = 0;
    for (const auto& e : w) inter_max = std::max(inter_max, e.first);
    auto pair_us = [&](int64_t p) { return (db.llen[static_cast<size_t>(2 * p)] + swk::kLanes - 1) * nch *
                                           step_us; };
    int64_t npipe = 0;
    if (nchp <= swk::kWavesPerWG) {
        if (db.opts->lpt_pipe >= 0) npipe = db.opts->lpt_pipe;
        else
            while (npipe < std::min<int64_t>(npairs, 4) && pair_us(npipe) > inter_max) ++npipe;
    }
    npipe = std::min(npipe, npairs);
    // The SHORTEST pairs in the pipelined form too (sw_opts lpt_pipe_tail n:
    // the last n pairs): the table ends with them, when the grid's slots
    // empty, and the pipeline cuts their latency to (length + 63 + 128
    // (chunks - 1)) steps of 2 rows per lane instead of (length + 63) of RI.
    // Default: 2 % of the pairs (to a multiple of 8) for linear scans of the
    // databases that run quads — measured on C2's 1/8 share under the
    // reference scoring (profiles/r06_tailpipe/): 12,794 / 12,802 / 12,803
    // -> 13,011 / 13,027 / 13,011 GCUPS with the last 32 of 1,561 pairs (16:
    // 13,018; 8, 24, 48, 64: 12,831, 12,879, 12,694, 12,772; 128 and more:
    // slower), affine scans within noise (their end is the tri groups').
    int64_t ntp = 0;
    if (db.opts->lpt_pipe_tail >= 0) ntp = db.opts->lpt_pipe_tail;
    else if (!affine && static_cast<double>(db.n) < kQuadMaxFill * kFillSubjects) ntp = (npairs * 2 / 100 + 4) / 8 * 8;
    if (nchp > swk::kWavesPerWG) ntp = 0;
    ntp = std::max<int64_t>(0, std::min(ntp, npairs - npipe));
    const int64_t pipe_tail = npairs - ntp;
    const int64_t npipe_wg = npipe / swk::kWavesPerWG;  // ordinary workgroups left with no pair
    for (int64_t g = npipe_wg; g < iwg; ++g) {
        const int64_t first = std::max<int64_t>(8 * g, 2 * npipe);  // its longest subject not pipelined
        if (first >= db.nlong || first >= 2 * pipe_tail) continue;
        w.emplace_back((db.llen[static_cast<size_t>(first)] + swk::kLanes - 1) * nch * step_us,
                       static_cast<int32_t>(-1 - g));
    }
    // (sw_scan_lpt item -1 - (iwg + pair)), ahead of everything
    for (int64_t p = 0; p < npipe; ++p) w.emplace_back(1e30 - p, static_cast<int32_t>(-1 - (iwg + p)));
    const double pstep_us = intra_step_us(2);
    for (int64_t p = pipe_tail; p < npairs; ++p)
        w.emplace_back((db.llen[static_cast<size_t>(2 * p)] + swk::kLanes - 1 + 128.0 * (nchp - 1)) * pstep_us,
                       static_cast<int32_t>(-1 - (iwg + p)));
    std::stable_sort(w.begin(), w.end(), [](const std::pair<double, int32_t>& x, const std::pair<double, int32_t>& y) {
        return x.first > y.first;
    });
    LptPlan out;
    out.order.resize(w.size());
    out.cost.resize(w.size());
    for (size_t k = 0; k < w.size(); ++k) {
        out.order[k] = w[k].second;
        out.cost[k] = static_cast<float>(w[k].first);
    }
    out.npipe = static_cast<int32_t>(npipe);
    out.pipe_tail = static_cast<int32_t>(pipe_tail);
    return out;
}

}  // namespace swplan
