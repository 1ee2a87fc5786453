// sw_plan.h — the host driver's scan-planning policies (sw_plan.cpp): plain
// functions of a read-only database view, so the policies and the merged
// launch's work table can be built and checked without a GPU
// (tests/test_plan.py).  sw_capi.cpp owns the databases and the device
// copies of the tables.
#pragma once

#include <cstdint>
#include <vector>

#include "sw_amd.h"

namespace swplan {

// What the policies read of a database (sw_capi.cpp sw_db).
struct PlanDb {
    int64_t n = 0;                        // subjects
    int64_t residues = 0;
    int64_t nblocks = 0;                  // 64-subject inter blocks
    int64_t nlong = 0;                    // long subjects (the wavefront kernel's)
    int32_t long_threshold = 0;
    const uint32_t* blk_groups = nullptr;  // [nblocks] 16-column groups per block, widest first
    const int32_t* llen = nullptr;         // [nlong] long subjects' lengths, longest first
    const sw_opts* opts = nullptr;         // the handle's kernel-form overrides
    int cus = 0;                           // the device's compute units
};

// Subjects longer than this go to the wavefront kernel (n, residues only).
int32_t default_long_threshold(const PlanDb& db);
// Leading (widest) blocks of the cooperative int32 kernel (divisor from the
// inter kernel's shape; 0 = none).
int32_t coop_blocks(const PlanDb& db, int divisor);
// Waves per group of the separate pair launch (2 or 4).
int pair_group(const PlanDb& db);
// Leading (widest) blocks of a two-strips scan run by wave groups.
int32_t pair_blocks(const PlanDb& db);
// The merged launch's widest group blocks by quads, or under affine gaps by
// 3-wave groups (0: none), and its narrowest blocks by pairs.
int32_t lpt_quad_blocks(const PlanDb& db, int32_t npair);
int32_t lpt_tri_blocks(const PlanDb& db, int32_t npair, int passes);
int32_t lpt_tail_blocks(const PlanDb& db, int32_t npair, int passes);
// Duration model (SIMD-busy microseconds and ticks of 8 columns of a pass).
double intra_step_us(int ri);
double single_ticks(int64_t ncols, int passes);
double group_ticks_host(int64_t ncols, int passes, int G);

// The merged launch's work table: entries longest (estimated) first.  An
// entry >= 0 is an inter workgroup of x2p_wg's numbering (groups, then
// single waves, then tail pairs); -1 - g an intra workgroup g (4 pairs) for
// g < iwg, or -1 - (iwg + p) pair p in the pipelined form (the longest
// npipe pairs and the pairs from pipe_tail on).
struct LptPlan {
    std::vector<int32_t> order;
    std::vector<float> cost;  // the estimate of each entry, microseconds
    int32_t npipe = 0;
    int32_t pipe_tail = 0;
};
LptPlan lpt_plan(const PlanDb& db, int32_t qpad, int rows, int32_t qpad_intra, int ri, int32_t npair, int32_t nquad,
                 int32_t ntail, bool affine, bool tri);

}  // namespace swplan
