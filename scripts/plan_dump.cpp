// scripts/plan_dump.cpp — the merged launch's work table (csrc/sw_plan.cpp
// lpt_plan) for a database shape given as files, for offline comparison of
// its duration estimates with a -DSW_TRACE_BLOCKS timeline
// (scripts/lpt_fit.py builds and runs it).
// usage: plan_dump GROUPS.u32 LLEN.i32 N RESIDUES QPAD ROWS QPAD_INTRA RI NPAIR NQUAD NTAIL AFFINE TRI OUT_PREFIX
// writes OUT_PREFIX.order (int32) and OUT_PREFIX.cost (float32), prints npipe and pipe_tail.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "sw_plan.h"

template <class T>
static std::vector<T> slurp(const char* path) {
    std::vector<T> v;
    FILE* f = std::fopen(path, "rb");
    if (!f) return v;
    T x;
    while (std::fread(&x, sizeof x, 1, f) == 1) v.push_back(x);
    std::fclose(f);
    return v;
}

int main(int argc, char** argv) {
    if (argc != 15) {
        std::fprintf(stderr, "usage: plan_dump GROUPS LLEN N RESIDUES QPAD ROWS QPAD_INTRA RI NPAIR NQUAD NTAIL AFFINE TRI OUT\n");
        return 2;
    }
    const std::vector<uint32_t> groups = slurp<uint32_t>(argv[1]);
    const std::vector<int32_t> llen = slurp<int32_t>(argv[2]);
    sw_opts o;
    std::memset(&o, 0, sizeof o);
    o.size = static_cast<int32_t>(sizeof o);
    for (int32_t* f : {&o.lpt_pipe, &o.quad_width, &o.pair_width, &o.pair_group, &o.coop_width, &o.tail_pairs,
                       &o.tri_width, &o.lpt_pipe_tail})
        *f = -1;
    swplan::PlanDb db;
    db.n = std::atoll(argv[3]);
    db.residues = std::atoll(argv[4]);
    db.nblocks = static_cast<int64_t>(groups.size());
    db.nlong = static_cast<int64_t>(llen.size());
    db.blk_groups = groups.data();
    db.llen = llen.data();
    db.opts = &o;
    db.cus = 256;
    db.long_threshold = swplan::default_long_threshold(db);
    const swplan::LptPlan p = swplan::lpt_plan(db, std::atoi(argv[5]), std::atoi(argv[6]), std::atoi(argv[7]),
                                               std::atoi(argv[8]), std::atoi(argv[9]), std::atoi(argv[10]),
                                               std::atoi(argv[11]), std::atoi(argv[12]) != 0, std::atoi(argv[13]) != 0);
    const std::string out = argv[14];
    FILE* f = std::fopen((out + ".order").c_str(), "wb");
    std::fwrite(p.order.data(), sizeof(int32_t), p.order.size(), f);
    std::fclose(f);
    f = std::fopen((out + ".cost").c_str(), "wb");
    std::fwrite(p.cost.data(), sizeof(float), p.cost.size(), f);
    std::fclose(f);
    std::printf("%d %d\n", p.npipe, p.pipe_tail);
    return 0;
}
