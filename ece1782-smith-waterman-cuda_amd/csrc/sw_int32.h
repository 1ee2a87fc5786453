// sw_int32.h — the int32 kernels' bodies (sw_kernels.hip): one 64-subject
// block per wave (inter_block, the recurrences of SWSolver.cu:246 / cpu.cpp
// with Gotoh's affine form) and one long subject per wave (intra_subject,
// the anti-diagonal wavefront).  In a header because the merged scan launch
// (sw_scan_lpt, sw_inter_x2.hip) runs them too: it re-scores, inside the same
// launch, the blocks and subjects its 16-bit cells flagged.
#pragma once

#include "sw_kernels.h"

namespace swk {

// LDS row stride (bytes) of the inter profile slice: >= R+16, a multiple of
// 16 with an odd number of 16-byte slots so that ds_read_b128 of different
// residue rows lands in different bank slots (MI355X_MICROARCH.md §LDS).
__host__ __device__ constexpr int inter_stride(int R) {
    return ((R + 16 + 15) / 16) % 2 == 1 ? ((R + 16 + 15) / 16) * 16
                                         : ((R + 16 + 15) / 16 + 1) * 16;
}

__device__ __forceinline__ int sx8(uint32_t w, int b) {
    return static_cast<int>(static_cast<int8_t>(w >> (8 * b)));
}

__device__ __forceinline__ int usub(int m, uint32_t g) {
    return static_cast<int>(__builtin_elementwise_sub_sat(static_cast<uint32_t>(m), g));
}

template <int N>
__device__ __forceinline__ uint32_t pword(const int4 (&v)[N], int w) {
    const int4 q = v[w >> 2];
    switch (w & 3) {
        case 0: return static_cast<uint32_t>(q.x);
        case 1: return static_cast<uint32_t>(q.y);
        case 2: return static_cast<uint32_t>(q.z);
        default: return static_cast<uint32_t>(q.w);
    }
}

// Stage rows [s0, s0+R) of the profile into the wave's LDS slice:
// 32 codes x R bytes = 2R chunks of 16 B, spread over the 64 lanes.
template <int R>
__device__ __forceinline__ void stage_profile(uint8_t* lp, const int8_t* __restrict__ prof,
                                              int stride, int s0, int lane) {
    constexpr int kChunks = kProfileRows * (R / 16);
    constexpr int S = inter_stride(R);
#pragma unroll
    for (int t = lane; t < kChunks; t += kLanes) {
        const int c = t / (R / 16);
        const int k = t % (R / 16);
        const int4 v = *reinterpret_cast<const int4*>(prof + static_cast<size_t>(c) * stride + s0 + 16 * k);
        *reinterpret_cast<int4*>(lp + c * S + 16 * k) = v;
    }
}

// ---------------------------------------------------------------------------
// inter-sequence kernels (linear and affine share one body)
// ---------------------------------------------------------------------------
// Per wave: one 64-subject block.  Per strip of R query rows: stage the
// profile slice, then walk the block's columns in sub-groups of SG columns.
// Software pipeline (the compiler would otherwise hoist every column's LDS
// reads and spill): the NEXT column's profile rows are read before the
// current column is computed, and the next sub-group's residues and boundary
// values are loaded at the top of the current sub-group; a sched_barrier
// closes each column.

template <int SG>
__device__ __forceinline__ void load_row(int (&v)[SG], const int32_t* p) {
#pragma unroll
    for (int q = 0; q < SG / 4; ++q) {
        const int4 t = *reinterpret_cast<const int4*>(p + 4 * q);
        v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
    }
}

template <int SG>
__device__ __forceinline__ void store_row(int32_t* p, const int (&v)[SG]) {
#pragma unroll
    for (int q = 0; q < SG / 4; ++q)
        *reinterpret_cast<int4*>(p + 4 * q) = make_int4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}

// `dep` ties the read to a value produced by the previous column: without it
// the IR scheduler hoists every unrolled column's LDS reads to the top of the
// body (sched_barrier only binds the machine scheduler) and the kernel
// balloons to 256+ VGPRs.
template <int R>
__device__ __forceinline__ void read_prof(int4 (&pv)[R / 16], const uint8_t* lp, uint32_t c, int dep) {
    constexpr int S = inter_stride(R);
    uint32_t off = c * S;
    asm volatile("" : "+v"(off) : "v"(dep));
    const int4* pp = reinterpret_cast<const int4*>(lp + off);
#pragma unroll
    for (int q = 0; q < R / 16; ++q) pv[q] = pp[q];
}

// One DP cell at row r of a lane's column (see the recurrences at the top).
// up: H of the cell above (in: row r-1, out: row r); diag: H(r-1, j-1) in,
// H(r, j-1) out; Hr/Er: this row's H and E (in: column j-1, out: column j,
// E already one column ahead); f: F one row ahead (affine).
template <bool AFFINE>
__device__ __forceinline__ void dp_cell(int& Hr, int& Er, int& up, int& f, int& diag, int sc, int& best,
                                        uint32_t go, uint32_t ge) {
    if constexpr (!AFFINE) {
        const int h = usub(max(max(Hr, up), diag + sc), go);
        diag = Hr;
        Hr = h;
        up = h;
        best = max(best, h);
    } else {
        const int h = max(max(Er, f), diag + sc);
        const int n = usub(h, go);
        Er = max(usub(Er, ge), n);
        f = max(usub(f, ge), n);
        diag = Hr;
        Hr = h;
        up = h;
        best = max(best, h);
    }
}

template <int R>
__device__ __forceinline__ int prof_at(const int4 (&p)[R / 16], int r) {
    return sx8(pword(p, r >> 2), r & 3);
}

// Walk the SG columns of one sub-group over the strip's R rows.
//   bh/bf  : in: H/F of the row above the strip (F one row ahead), per column;
//            out: the strip's bottom row H/F, per column.
//   dtop   : H(s0-1, first column - 1); out: H(s0-1, last column).
//   pa, pb : in: profile rows of columns 0 (and 1 with SKEW); out, if `more`:
//            those of rs_next's first columns (software pipeline; `dep`-tied
//            reads so the compiler cannot hoist them all and spill).
// SKEW: columns are taken in pairs, cell (r, j) beside cell (r-1, j+1): two
// independent dependency chains per step, so the 3-deep affine chain (max3,
// sub, max through F) and the 2-deep linear one hide their latency at the 2-3
// waves per SIMD the register budget allows (profiles/r01_chain_rate.txt).
template <int R, int SG, bool AFFINE, bool SKEW>
__device__ __forceinline__ void sweep_group(int (&H)[R], int (&E)[AFFINE ? R : 1], int (&bh)[SG],
                                            int (&bf)[AFFINE ? SG : 1], int& dtop, int& best, const uint8_t* lp,
                                            const Residues<SG>& rs, const Residues<SG>& rs_next, bool more,
                                            int4 (&pa)[R / 16], int4 (&pb)[R / 16], uint32_t go, uint32_t ge) {
    if constexpr (!SKEW) {
#pragma unroll
        for (int jj = 0; jj < SG; ++jj) {
            int4 pn[R / 16];
            if (jj + 1 < SG) {
                read_prof<R>(pn, lp, rs.code(jj + 1), H[R - 1]);
            } else if (more) {
                read_prof<R>(pn, lp, rs_next.code(0), H[R - 1]);
            }
            int up = bh[jj];
            int diag = dtop;
            dtop = up;
            int f = AFFINE ? bf[AFFINE ? jj : 0] : 0;
#pragma unroll
            for (int r = 0; r < R; ++r)
                dp_cell<AFFINE>(H[r], E[AFFINE ? r : 0], up, f, diag, prof_at<R>(pa, r), best, go, ge);
            bh[jj] = up;
            if constexpr (AFFINE) bf[jj] = f;
            if (jj + 1 < SG || more) {
#pragma unroll
                for (int q = 0; q < R / 16; ++q) pa[q] = pn[q];
            }
            // Stop LLVM from reassociating the running max across the
            // unrolled columns (it would keep every column's H alive).
            asm volatile("" : "+v"(best));
            __builtin_amdgcn_sched_barrier(0);
        }
    } else {
        static_assert(SG % 2 == 0, "column pairs");
#pragma unroll
        for (int jj = 0; jj < SG; jj += 2) {
            int4 na[R / 16], nb[R / 16];
            if (jj + 2 < SG) {
                read_prof<R>(na, lp, rs.code(jj + 2), H[R - 1]);
                read_prof<R>(nb, lp, rs.code(jj + 3), H[R - 1]);
            } else if (more) {
                read_prof<R>(na, lp, rs_next.code(0), H[R - 1]);
                read_prof<R>(nb, lp, rs_next.code(1), H[R - 1]);
            }
            int upA = bh[jj], upB = bh[jj + 1];
            int diagA = dtop, diagB = upA;
            dtop = upB;
            int fA = AFFINE ? bf[AFFINE ? jj : 0] : 0;
            int fB = AFFINE ? bf[AFFINE ? jj + 1 : 0] : 0;
            dp_cell<AFFINE>(H[0], E[0], upA, fA, diagA, prof_at<R>(pa, 0), best, go, ge);
#pragma unroll
            for (int r = 1; r < R; ++r) {
                dp_cell<AFFINE>(H[r], E[AFFINE ? r : 0], upA, fA, diagA, prof_at<R>(pa, r), best, go, ge);
                dp_cell<AFFINE>(H[r - 1], E[AFFINE ? r - 1 : 0], upB, fB, diagB, prof_at<R>(pb, r - 1), best, go,
                                ge);
            }
            dp_cell<AFFINE>(H[R - 1], E[AFFINE ? R - 1 : 0], upB, fB, diagB, prof_at<R>(pb, R - 1), best, go, ge);
            bh[jj] = upA;
            bh[jj + 1] = upB;
            if constexpr (AFFINE) {
                bf[jj] = fA;
                bf[jj + 1] = fB;
            }
            if (jj + 2 < SG || more) {
#pragma unroll
                for (int q = 0; q < R / 16; ++q) {
                    pa[q] = na[q];
                    pb[q] = nb[q];
                }
            }
            asm volatile("" : "+v"(best));
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

template <int R, int SG, bool AFFINE, bool SKEW>
__device__ __forceinline__ void inter_block(const InterArgs& a, int blk, uint8_t* lp, int lane) {
    const uint32_t ncols = a.blk_groups[blk] * kGroupCols;
    const uint64_t base = a.blk_off[blk] + static_cast<uint64_t>(lane) * kGroupCols;
    const uint32_t go = static_cast<uint32_t>(a.gap_open);
    const uint32_t ge = static_cast<uint32_t>(a.gap_extend);
    int best = 0;
    if (ncols == 0) goto done;

    for (int s0 = 0; s0 < a.qpad; s0 += R) {
        const bool first = (s0 == 0);
        const bool last = (s0 + R >= a.qpad);
        stage_profile<R>(lp, a.prof, a.prof_stride, s0, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");

        int H[R];
        int E[AFFINE ? R : 1];
#pragma unroll
        for (int r = 0; r < R; ++r) H[r] = 0;
#pragma unroll
        for (int r = 0; r < (AFFINE ? R : 1); ++r) E[r] = 0;
        int dtop = 0;  // H(s0-1, j-1)

        Residues<SG> rs, rs_next;
        int bh[SG], bh_next[SG];
        int bf[AFFINE ? SG : 1], bf_next[AFFINE ? SG : 1];
        rs.load(a.residues + base);
        if (!first) {
            load_row<SG>(bh, a.bnd_h + base);
            if constexpr (AFFINE) load_row<SG>(bf, a.bnd_f + base);
        } else {
#pragma unroll
            for (int q = 0; q < SG; ++q) bh[q] = 0;
#pragma unroll
            for (int q = 0; q < (AFFINE ? SG : 1); ++q) bf[q] = 0;
        }
        int4 pa[R / 16], pb[R / 16];
        read_prof<R>(pa, lp, rs.code(0), 0);
        if constexpr (SKEW) read_prof<R>(pb, lp, rs.code(1), 0);

        for (uint32_t col0 = 0; col0 < ncols; col0 += SG) {
            const uint64_t idx = base + (col0 >> 4) * kGroupBytes + (col0 & 15);
            const bool more = col0 + SG < ncols;
            const uint64_t nidx = base + ((col0 + SG) >> 4) * kGroupBytes + ((col0 + SG) & 15);
            if (more) {
                rs_next.load(a.residues + nidx);
                if (!first) {
                    load_row<SG>(bh_next, a.bnd_h + nidx);
                    if constexpr (AFFINE) load_row<SG>(bf_next, a.bnd_f + nidx);
                }
            }
            sweep_group<R, SG, AFFINE, SKEW>(H, E, bh, bf, dtop, best, lp, rs, rs_next, more, pa, pb, go, ge);
            if (!last) {
                store_row<SG>(a.bnd_h + idx, bh);
                if constexpr (AFFINE) store_row<SG>(a.bnd_f + idx, bf);
            }
            if (more) {
                rs = rs_next;
                if (!first) {
#pragma unroll
                    for (int q = 0; q < SG; ++q) bh[q] = bh_next[q];
                    if constexpr (AFFINE) {
#pragma unroll
                        for (int q = 0; q < SG; ++q) bf[q] = bf_next[q];
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < SG; ++q) bh[q] = 0;
                    if constexpr (AFFINE) {
#pragma unroll
                        for (int q = 0; q < SG; ++q) bf[q] = 0;
                    }
                }
            }
        }
    }
done:
    const int id = a.lane_ids[static_cast<size_t>(blk) * kLanes + lane];
    if (id >= 0) a.scores[id] = best;
}

// DPP controls (GFX9 family): wave_shr:1 moves lane t-1's value to lane t;
// lane 0 keeps `old`.
constexpr int kDppWaveShr1 = 0x138;

__device__ __forceinline__ int shr1(int old, int src) {
    return __builtin_amdgcn_update_dpp(old, src, kDppWaveShr1, 0xf, 0xf, false);
}

// Per-lane slot of RIP = RI rounded up to 4 bytes (intra_rip, sw_kernels.h);
// the host lays the intra profile out as [chunk][code][lane][RIP] so staging
// is a straight copy.
// +4 bytes per code row: lanes reading different codes start on different banks
__host__ __device__ constexpr int intra_stride(int RI) { return kLanes * intra_rip(RI) + 4; }

// WG: the subject's wave is its workgroup (sw_intra: 64 threads), so the
// LDS staging synchronises with workgroup barriers; otherwise (the merged
// launch, one wave of a 256-thread workgroup) with wave barriers.
template <int RI, bool AFFINE, bool WG = true>
__device__ __forceinline__ void intra_subject(const IntraArgs& a, int sid, uint8_t* lds) {
    auto sync = [] {
        if constexpr (WG) {
            __syncthreads();
        } else {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
    };
    constexpr int CH = kLanes * RI;  // query rows per chunk
    constexpr int RIP = intra_rip(RI);
    constexpr int S = intra_stride(RI);
    constexpr int CHUNK_BYTES = kProfileRows * kLanes * RIP;  // one chunk of the host profile
    const int lane = threadIdx.x & (kLanes - 1);
    const int L = a.subj_len[sid];
    const uint8_t* __restrict__ res = a.residues + a.subj_off[sid];
    int32_t* bnd_h = a.bnd_h + a.subj_off[sid];
    int32_t* bnd_f = AFFINE ? a.bnd_f + a.subj_off[sid] : nullptr;
    const uint32_t go = static_cast<uint32_t>(a.gap_open);
    const uint32_t ge = static_cast<uint32_t>(a.gap_extend);
    int best = 0;

    for (int c0 = 0, ch = 0; c0 < a.qpad; c0 += CH, ++ch) {
        const bool first = (c0 == 0);
        const bool last = (c0 + CH >= a.qpad);
        sync();  // previous chunk's LDS reads are done
        // stage this chunk's profile: [code][lane][RIP] -> rows of S bytes
        const int8_t* src = a.prof + static_cast<size_t>(ch) * CHUNK_BYTES;
        for (int t = lane; t < CHUNK_BYTES / 16; t += kLanes) {
            const int c = t / (kLanes * RIP / 16);
            const int k = t % (kLanes * RIP / 16);
            const int4 v = *reinterpret_cast<const int4*>(src + 16 * t);
            int* d = reinterpret_cast<int*>(lds + c * S + 16 * k);  // S is 4-byte aligned only
            d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        }
        sync();

        int H[RI], E[AFFINE ? RI : 1];
#pragma unroll
        for (int r = 0; r < RI; ++r) H[r] = 0;
#pragma unroll
        for (int r = 0; r < (AFFINE ? RI : 1); ++r) E[r] = 0;
        int hl = 0, fl = 0;         // this lane's bottom row H, F at its last column
        int up_prev = 0;            // H of the row above at column j-1 (diag of row 0)
        int rc = kPadCode;          // residue code of this lane's current column
        int in_res = kPadCode, in_bh = 0, in_bf = 0, out_h = 0, out_f = 0;
        const int nsteps = L + kLanes - 1;
        const uint8_t* lrow = lds + lane * RIP;

        for (int k0 = 0; k0 < nsteps; k0 += kLanes) {
            // refill lane-0 conveyors for steps k0..k0+63 (column k = step)
            {
                const int col = k0 + lane;
                in_res = col < L ? res[col] : kPadCode;
                in_bh = (!first && col < L) ? bnd_h[col] : 0;
                if (AFFINE) in_bf = (!first && col < L) ? bnd_f[col] : 0;
            }
            const int mend = min(kLanes, nsteps - k0);
            for (int m = 0; m < mend; ++m) {
                const int sres = __builtin_amdgcn_readlane(in_res, m);
                const int sbh = __builtin_amdgcn_readlane(in_bh, m);
                rc = shr1(sres, rc);
                const int up0 = shr1(sbh, hl);
                int f = 0;
                if (AFFINE) {
                    const int sbf = __builtin_amdgcn_readlane(in_bf, m);
                    f = shr1(sbf, fl);
                }
                const uint32_t* pp = reinterpret_cast<const uint32_t*>(lrow + rc * S);
                uint32_t pw[RIP / 4];
#pragma unroll
                for (int q = 0; q < RIP / 4; ++q) pw[q] = pp[q];
                int up = up0;
                int diag = up_prev;
                up_prev = up0;
#pragma unroll
                for (int r = 0; r < RI; ++r) {
                    const int sc = sx8(pw[r >> 2], r & 3);
                    int h;
                    if (AFFINE) {
                        const int e = max(usub(E[r], ge), usub(H[r], go));
                        f = max(usub(f, ge), usub(up, go));
                        h = max(max(e, f), diag + sc);
                        E[r] = e;
                    } else {
                        h = usub(max(max(H[r], up), diag + sc), go);
                    }
                    diag = H[r];
                    H[r] = h;
                    up = h;
                    best = max(best, h);
                }
                hl = up;
                fl = f;
                if (!last) {
                    // lane 63 finished column k - 63: collect it for the next chunk
                    const int k = k0 + m;
                    const int oc = k - (kLanes - 1);
                    if (oc >= 0) {
                        const int slot = oc & (kLanes - 1);
                        const bool mine = (lane == slot);
                        const int vh = __builtin_amdgcn_readlane(hl, kLanes - 1);
                        out_h = mine ? vh : out_h;
                        if (AFFINE) {
                            const int vf = __builtin_amdgcn_readlane(fl, kLanes - 1);
                            out_f = mine ? vf : out_f;
                        }
                        if (slot == kLanes - 1 || oc == L - 1) {
                            const int col = (oc & ~(kLanes - 1)) + lane;
                            if (col <= oc) {
                                bnd_h[col] = out_h;
                                if (AFFINE) bnd_f[col] = out_f;
                            }
                        }
                    }
                }
            }
        }
    }
    // wave max-reduction of best
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) best = max(best, __shfl_xor(best, off));
    if (lane == 0) a.scores[a.subj_id[sid]] = best;
    sync();  // list mode: the next subject restages the LDS profile
}

}  // namespace swk
