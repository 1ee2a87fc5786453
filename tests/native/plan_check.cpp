// tests/native/plan_check.cpp — CPU check of the merged launch's work table
// (sw_plan.cpp lpt_plan) against the kernel's decoding of it
// (sw_inter_x2.hip x2p_wg and sw_scan_lpt, sw_intra_x2.h intra_x2_wg):
// every inter block and every long-subject pair is scanned by exactly one
// entry, whatever mix of quads / tri groups with spare waves / pairs /
// single waves / tail pairs and pipelined pairs the policies choose, and the
// table is sorted longest first.  Built and run by tests/test_plan.py.
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "sw_kernels.h"
#include "sw_plan.h"

static int failures = 0;
#define CHECK(c, ...)                          \
    do {                                       \
        if (!(c)) {                            \
            std::printf("FAIL: " __VA_ARGS__); \
            std::printf("\n");                 \
            ++failures;                        \
        }                                      \
    } while (0)

// one scenario: nb blocks of widths decreasing from wmax to wmin (16-column
// groups), nlong long subjects of lengths decreasing from lmax to lmax / 2
static void scenario(const char* name, int64_t nb, int wmax, int wmin, int64_t nlong, int lmax, int32_t npair,
                     int32_t nquad, int32_t ntail, bool affine, bool tri, int qlen, int rows, int ri, sw_opts o) {
    std::vector<uint32_t> groups(nb);
    for (int64_t b = 0; b < nb; ++b)
        groups[b] = static_cast<uint32_t>((wmax - (wmax - wmin) * b / (nb > 1 ? nb - 1 : 1) + 15) / 16);
    std::vector<int32_t> llen(nlong);
    for (int64_t k = 0; k < nlong; ++k) llen[k] = static_cast<int32_t>(lmax - (lmax / 2) * k / (nlong > 1 ? nlong - 1 : 1));
    swplan::PlanDb db;
    db.n = nb * 64 + nlong;
    db.residues = db.n * 300;
    db.nblocks = nb;
    db.nlong = nlong;
    db.long_threshold = lmax / 2;
    db.blk_groups = groups.data();
    db.llen = llen.data();
    db.opts = &o;
    db.cus = 256;
    const int32_t qpad = (qlen + rows - 1) / rows * rows;
    const int32_t qpad_intra = (qlen + 64 * ri - 1) / (64 * ri) * (64 * ri);
    const swplan::LptPlan p = swplan::lpt_plan(db, qpad, rows, qpad_intra, ri, npair, nquad, ntail, affine, tri);
    // the kernel's decoding (x2p_wg: MERGED, GMAX 4)
    const int64_t pwg = nquad + (npair - nquad + 1) / 2;
    const int64_t tail = ntail > 0 && nb - ntail > npair && nb - ntail < nb ? nb - ntail : nb;
    const bool tri_on = tri && affine;
    const int64_t nspare = tri_on ? std::max<int64_t>(0, std::min<int64_t>(nquad, tail - npair)) : 0;
    const int64_t s0 = npair + nspare;
    const int64_t twg = pwg + (tail - s0 + swk::kWavesPerWG - 1) / swk::kWavesPerWG;
    const int64_t npairs = (nlong + 1) / 2;
    const int64_t niwg = (npairs + swk::kWavesPerWG - 1) / swk::kWavesPerWG;
    std::vector<int> blk_seen(nb, 0), pair_seen(npairs, 0);
    std::vector<int> entry_seen(p.order.size() + 16, 0);
    for (size_t k = 0; k < p.order.size(); ++k) {
        const int32_t it = p.order[k];
        if (k) CHECK(p.cost[k] <= p.cost[k - 1], "%s: entry %zu out of order", name, k);
        if (it >= 0) {
            const int64_t wgi = it;
            if (wgi >= pwg && wgi < twg) {  // single waves
                for (int w = 0; w < swk::kWavesPerWG; ++w) {
                    const int64_t b = s0 + (wgi - pwg) * swk::kWavesPerWG + w;
                    if (b < tail) ++blk_seen[b];
                }
            } else if (wgi >= twg) {        // tail pairs: two blocks
                for (int q = 0; q < 2; ++q) {
                    const int64_t b = tail + (wgi - twg) * 2 + q;
                    if (b < nb) ++blk_seen[b];
                }
            } else if (wgi < nquad) {       // a quad or a tri (+ its spare's single)
                ++blk_seen[wgi];
                if (tri_on && npair + wgi < s0) ++blk_seen[npair + wgi];
            } else {                        // pairs: two blocks
                for (int q = 0; q < 2; ++q) {
                    const int64_t b = nquad + (wgi - nquad) * 2 + q;
                    if (b < npair) ++blk_seen[b];
                }
            }
        } else {
            const int64_t g = -1 - static_cast<int64_t>(it);
            if (g < niwg) {                 // an intra workgroup: pairs 4g .. 4g + 3, minus the pipelined
                for (int w = 0; w < swk::kWavesPerWG; ++w) {
                    const int64_t pr = g * swk::kWavesPerWG + w;
                    if (pr < npairs && pr >= p.npipe && pr < p.pipe_tail) ++pair_seen[pr];
                }
            } else {                        // a pipelined pair
                const int64_t pr = g - niwg;
                CHECK(pr >= 0 && pr < npairs, "%s: pipelined pair %lld out of range", name, (long long)pr);
                CHECK(pr < p.npipe || pr >= p.pipe_tail, "%s: pair %lld pipelined but not in a pipelined range", name,
                      (long long)pr);
                if (pr >= 0 && pr < npairs) ++pair_seen[pr];
            }
        }
    }
    for (int64_t b = 0; b < nb; ++b) CHECK(blk_seen[b] == 1, "%s: block %lld scanned %d times", name, (long long)b, blk_seen[b]);
    for (int64_t pr = 0; pr < npairs; ++pr)
        CHECK(pair_seen[pr] == 1, "%s: pair %lld scanned %d times", name, (long long)pr, pair_seen[pr]);
    std::printf("%s: %zu entries, npipe %d, pipe_tail %d of %lld pairs, spares %lld\n", name, p.order.size(), p.npipe,
                p.pipe_tail, (long long)npairs, (long long)nspare);
}

// the library's choice for every policy (sw_opts_init's -1s; the checker
// links sw_plan.cpp alone)
static sw_opts policy_defaults() {
    sw_opts o;
    std::memset(&o, 0, sizeof o);
    o.size = static_cast<int32_t>(sizeof o);
    for (int32_t* f : {&o.lpt_pipe, &o.quad_width, &o.pair_width, &o.pair_group, &o.coop_width, &o.tail_pairs,
                       &o.tri_width, &o.lpt_pipe_tail})
        *f = -1;
    return o;
}

int main() {
    const sw_opts o = policy_defaults();
    // C2's 1/8 share shape: 1,065 blocks, 3,122 long subjects, 375-aa query
    scenario("share8-affine-tri", 1065, 891, 32, 3122, 7429, 633, 275, 0, true, true, 375, 64, 6, o);
    scenario("share8-affine-quads", 1065, 891, 32, 3122, 7429, 633, 105, 0, true, false, 375, 64, 6, o);
    scenario("share8-linear-tailpipe", 1065, 891, 32, 3122, 7429, 633, 105, 0, false, false, 375, 96, 6, o);
    // more tris than single blocks: spares run out
    scenario("tris-exceed-singles", 200, 800, 100, 40, 2000, 190, 190, 0, true, true, 375, 64, 6, o);
    // tail pairs beside tris
    scenario("tris-and-tail-pairs", 2000, 1500, 16, 500, 4000, 600, 100, 256, true, true, 300, 64, 4, o);
    // a tail-pair count reaching into the group blocks: the kernel runs none
    scenario("tail-pairs-clamped", 300, 900, 48, 80, 3000, 250, 20, 100, true, true, 375, 64, 6, o);
    // forced pipes at both ends, odd long count
    sw_opts f = o;
    f.lpt_pipe = 3;
    f.lpt_pipe_tail = 37;
    scenario("pipes-both-ends", 500, 900, 48, 301, 5000, 300, 50, 64, true, true, 375, 64, 6, f);
    f.lpt_pipe_tail = 100000;  // every pair pipelined
    scenario("every-pair-pipelined", 300, 700, 48, 120, 3000, 150, 0, 0, false, false, 200, 64, 4, f);
    // no long subjects, no groups
    scenario("inter-only", 50, 300, 16, 0, 0, 0, 0, 0, true, false, 375, 64, 6, o);
    if (failures) {
        std::printf("%d failures\n", failures);
        return 1;
    }
    std::printf("plan_check ok\n");
    return 0;
}
