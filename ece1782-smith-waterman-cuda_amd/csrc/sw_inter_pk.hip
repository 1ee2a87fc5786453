// sw_inter_pk.hip — inter-sequence Smith-Waterman, two subjects per lane,
// packed 16-bit cells.
//
// Why: the scan is bound by VALU instructions per cell.  The int32 cell needs
// ~3.5 instructions, most of them issuing at the slow ~4.2-cycle rate on
// gfx950; a packed-16 cell (v_pk_add_u16, 2 x v_pk_max_i16, v_pk_sub_u16
// clamp, v_pk_max_i16 for the running maximum) does TWO cells in 5
// instructions.  A faithful dependent-chain microbenchmark measured it
// 1.13-1.25x faster per cell (profiles/r01_chain_rate.txt).  Packing pays only
// if the pair of scores (S[q_i][a], S[q_i][b]) for the two subjects' residues
// a, b arrives in one register without a v_perm/v_bfi: each strip the
// workgroup builds a PAIR TABLE in LDS, entry (a, b) holding R rows of
// (S[q_i][a] | S[q_i][b] << 16); a lane reads its column's entry with
// ds_read_b128.
//
// Layout: wave w of workgroup g handles blocks 2p and 2p+1 (p = g*WPG + w) of
// the packed database (sw_capi.cpp): lane l's low half is subject (2p, l), its
// high half subject (2p+1, l).  Blocks are sorted longest-first, so 2p is the
// wider one; columns past block 2p+1's width read as the zero-score pad code.
// Strip boundary rows are packed pairs in block 2p's slot of the int32
// boundary array.  The WPG waves of a workgroup walk the query strips in step
// (one table per strip, three barriers per strip).
//
// Values live in 0..32767; a half whose running maximum reaches kSat16 may
// have overflowed, and its block goes on the rescue list for the int32 kernel.
#include "sw_kernels.h"

namespace swk {

typedef short s2 __attribute__((ext_vector_type(2)));
typedef unsigned short u2 __attribute__((ext_vector_type(2)));

constexpr int kPkCodes = 26;                    // residue codes 0..24 + pad (25)
constexpr int kPkEntries = kPkCodes * kPkCodes;  // (a, b) pairs

__host__ __device__ constexpr int pk_entry_stride(int R) {
    // R*4 bytes + 16, with an odd number of 16-byte slots (bank spread)
    return ((R * 4 + 16) / 16) % 2 == 1 ? R * 4 + 16 : R * 4 + 32;
}
__host__ __device__ constexpr int pk_lds_bytes(int R) {
    return kPkEntries * pk_entry_stride(R) + kPkCodes * R * 2;
}

__device__ __forceinline__ s2 as_s2(uint32_t x) { return __builtin_bit_cast(s2, x); }
__device__ __forceinline__ uint32_t as_u32(s2 x) { return __builtin_bit_cast(uint32_t, x); }

template <int SG>
struct PkResidues {  // the two subjects' codes for SG columns
    uint32_t a[SG / 4], b[SG / 4];
    __device__ __forceinline__ uint32_t code(const uint32_t* w, int jj) const {
        return (w[jj >> 2] >> (8 * (jj & 3))) & 0xffu;
    }
    __device__ __forceinline__ uint32_t entry(int jj) const { return code(a, jj) * kPkCodes + code(b, jj); }
};

template <int SG>
__device__ __forceinline__ void load_codes(uint32_t (&w)[SG / 4], const uint8_t* p, bool valid) {
    if (valid) {
        if constexpr (SG == 4) {
            w[0] = *reinterpret_cast<const uint32_t*>(p);
        } else if constexpr (SG == 8) {
            const int2 v = *reinterpret_cast<const int2*>(p);
            w[0] = v.x; w[1] = v.y;
        } else {
            const int4 v = *reinterpret_cast<const int4*>(p);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < SG / 4; ++q) w[q] = 0x19191919u;  // kPadCode in every byte
    }
}

// `dep` ties the read to a value of the previous chunk so the scheduler
// cannot hoist every unrolled read to the top of the loop body.
__device__ __forceinline__ void read_pairs(int4 (&p)[4], const uint8_t* tbl, uint32_t off, uint32_t dep) {
    asm volatile("" : "+v"(off) : "v"(dep));
    const int4* pp = reinterpret_cast<const int4*>(tbl + off);
    p[0] = pp[0];
    p[1] = pp[1];
    p[2] = pp[2];
    p[3] = pp[3];
}

template <int R, int SG, int WPG>
__global__ __launch_bounds__(64 * WPG) void sw_inter_pk(InterArgs a) {
    static_assert(R % 16 == 0 && SG % 4 == 0, "shape");
    constexpr int ES = pk_entry_stride(R);
    constexpr int NCH = R / 16;  // 16-row chunks per column (4 x ds_read_b128)
    constexpr int STEPS = SG * NCH;
    extern __shared__ __attribute__((aligned(16))) uint8_t pk_lds[];
    uint8_t* tbl = pk_lds;
    int16_t* sprof = reinterpret_cast<int16_t*>(pk_lds + kPkEntries * ES);

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int npairs = (a.nblocks + 1) / 2;
    const int pair = blockIdx.x * WPG + wave;
    const bool active = pair < npairs;
    const int b0 = 2 * pair;
    const int b1 = 2 * pair + 1;
    const bool has1 = active && b1 < a.nblocks;
    const uint32_t ncols = active ? a.blk_groups[b0] * kGroupCols : 0;
    const uint32_t ncols1 = has1 ? a.blk_groups[b1] * kGroupCols : 0;
    const uint64_t base0 = active ? a.blk_off[b0] + static_cast<uint64_t>(lane) * kGroupCols : 0;
    const uint64_t base1 = has1 ? a.blk_off[b1] + static_cast<uint64_t>(lane) * kGroupCols : 0;
    const int16_t* prof16 = reinterpret_cast<const int16_t*>(a.prof);
    uint32_t* bnd = reinterpret_cast<uint32_t*>(a.bnd_h);
    const u2 g2 = {static_cast<unsigned short>(a.gap_open), static_cast<unsigned short>(a.gap_open)};
    s2 best = {0, 0};

    for (int s0 = 0; s0 < a.qpad; s0 += R) {
        const bool first = (s0 == 0);
        const bool last = (s0 + R >= a.qpad);
        // ---- this strip's pair table (all waves of the workgroup) ----
        __syncthreads();  // the previous strip's table is no longer read
        for (int t = threadIdx.x; t < kPkCodes * R; t += 64 * WPG) {
            const int c = t / R, r = t % R;
            sprof[c * R + r] = prof16[static_cast<size_t>(c) * a.prof_stride + s0 + r];
        }
        __syncthreads();
        for (int t = threadIdx.x; t < kPkEntries * R; t += 64 * WPG) {
            const int e = t / R, r = t % R;
            const int ca = e / kPkCodes, cb = e % kPkCodes;
            const uint32_t v = static_cast<uint16_t>(sprof[ca * R + r]) |
                               (static_cast<uint32_t>(static_cast<uint16_t>(sprof[cb * R + r])) << 16);
            *reinterpret_cast<uint32_t*>(tbl + e * ES + 4 * r) = v;
        }
        __syncthreads();
        if (ncols == 0) continue;  // wave-uniform: idle waves still join every barrier

        s2 H[R];
#pragma unroll
        for (int r = 0; r < R; ++r) H[r] = s2{0, 0};
        s2 dtop = {0, 0};

        PkResidues<SG> rs, rs_next;
        uint32_t bw[SG], bw_next[SG];
        load_codes<SG>(rs.a, a.residues + base0, true);
        load_codes<SG>(rs.b, a.residues + base1, ncols1 > 0);
        if (!first) {
#pragma unroll
            for (int q = 0; q < SG / 4; ++q) {
                const int4 v = *reinterpret_cast<const int4*>(bnd + base0 + 4 * q);
                bw[4 * q] = v.x; bw[4 * q + 1] = v.y; bw[4 * q + 2] = v.z; bw[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int q = 0; q < SG; ++q) bw[q] = 0;
        }
        int4 P[2][4];
        read_pairs(P[0], tbl, rs.entry(0) * ES, 0);

        for (uint32_t col0 = 0; col0 < ncols; col0 += SG) {
            const uint64_t off = (col0 >> 4) * kGroupBytes + (col0 & 15);
            const bool more = col0 + SG < ncols;
            const uint32_t ncol = col0 + SG;
            const uint64_t noff = (ncol >> 4) * kGroupBytes + (ncol & 15);
            if (more) {
                load_codes<SG>(rs_next.a, a.residues + base0 + noff, true);
                load_codes<SG>(rs_next.b, a.residues + base1 + noff, ncol < ncols1);
                if (!first) {
#pragma unroll
                    for (int q = 0; q < SG / 4; ++q) {
                        const int4 v = *reinterpret_cast<const int4*>(bnd + base0 + noff + 4 * q);
                        bw_next[4 * q] = v.x; bw_next[4 * q + 1] = v.y;
                        bw_next[4 * q + 2] = v.z; bw_next[4 * q + 3] = v.w;
                    }
                }
            }
            s2 up = {0, 0}, diag = {0, 0};
#pragma unroll
            for (int t = 0; t < STEPS; ++t) {
                const int jj = t / NCH;
                const int k = t % NCH;
                if (t + 1 < STEPS) {
                    const int jn = (t + 1) / NCH, kn = (t + 1) % NCH;
                    read_pairs(P[(t + 1) & 1], tbl, rs.entry(jn) * ES + 64 * kn,
                               as_u32(k == 0 ? H[R - 1] : H[16 * k - 1]));
                } else if (more) {
                    read_pairs(P[(t + 1) & 1], tbl, rs_next.entry(0) * ES, as_u32(H[16 * k - 1]));
                }
                if (k == 0) {
                    up = as_s2(bw[jj]);
                    diag = dtop;
                    dtop = up;
                }
                const int4(&pc)[4] = P[t & 1];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t pw[4] = {static_cast<uint32_t>(pc[q].x), static_cast<uint32_t>(pc[q].y),
                                            static_cast<uint32_t>(pc[q].z), static_cast<uint32_t>(pc[q].w)};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int r = 16 * k + 4 * q + e;
                        const s2 av = diag + as_s2(pw[e]);
                        const s2 m = __builtin_elementwise_max(__builtin_elementwise_max(H[r], up), av);
                        const s2 h = __builtin_bit_cast(
                            s2, __builtin_elementwise_sub_sat(__builtin_bit_cast(u2, m), g2));
                        diag = H[r];
                        H[r] = h;
                        up = h;
                        best = __builtin_elementwise_max(best, h);
                    }
                }
                if (k == NCH - 1) {
                    bw[jj] = as_u32(up);  // bottom row of this strip, column col0 + jj
                    asm volatile("" : "+v"(best));
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            if (!last) {
#pragma unroll
                for (int q = 0; q < SG / 4; ++q)
                    *reinterpret_cast<int4*>(bnd + base0 + off + 4 * q) =
                        make_int4(static_cast<int>(bw[4 * q]), static_cast<int>(bw[4 * q + 1]),
                                  static_cast<int>(bw[4 * q + 2]), static_cast<int>(bw[4 * q + 3]));
            }
            if (more) {
                rs = rs_next;
#pragma unroll
                for (int q = 0; q < SG; ++q) bw[q] = first ? 0u : bw_next[q];
            }
        }
    }
    if (active) {
        const int lo = best.x, hi = best.y;  // sign-extended halves
        const bool sat0 = lo >= kSat16 || lo < 0;
        const bool sat1 = hi >= kSat16 || hi < 0;
        const int id0 = a.lane_ids[static_cast<size_t>(b0) * kLanes + lane];
        if (id0 >= 0) a.scores[id0] = lo < 0 ? 0 : lo;
        if (has1) {
            const int id1 = a.lane_ids[static_cast<size_t>(b1) * kLanes + lane];
            if (id1 >= 0) a.scores[id1] = hi < 0 ? 0 : hi;
        }
        const uint64_t m0 = __builtin_amdgcn_ballot_w64(sat0);
        const uint64_t m1 = __builtin_amdgcn_ballot_w64(sat1);
        if (lane == 0) {
            if (m0) a.rescue_list[atomicAdd(a.rescue_count, 1)] = b0;
            if (m1 && has1) a.rescue_list[atomicAdd(a.rescue_count, 1)] = b1;
        }
    }
}

template <int R, int SG, int WPG>
static hipError_t launch_pk_shape(const InterArgs& a, hipStream_t s) {
    const int npairs = (a.nblocks + 1) / 2;
    const dim3 grid((npairs + WPG - 1) / WPG);
    const size_t lds = pk_lds_bytes(R);
    static bool attr_set = false;  // >64 KiB dynamic LDS must be opted into
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&sw_inter_pk<R, SG, WPG>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    hipLaunchKernelGGL((sw_inter_pk<R, SG, WPG>), grid, dim3(64 * WPG), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_inter_pk(const InterArgs& a, int R, int SG, hipStream_t s) {
    if (a.nblocks <= 0 || a.qpad <= 0) return hipSuccess;
    // SG == 8 / 16: 4-wave workgroups (fine-grained work units); SG == 9 is
    // encoded by the tuning string "k16x9" = 16-wave workgroups, SG 8.
    if (R == 16 && SG == 8) return launch_pk_shape<16, 8, 4>(a, s);
    if (R == 16 && SG == 16) return launch_pk_shape<16, 16, 4>(a, s);
    if (R == 16 && SG == 9) return launch_pk_shape<16, 8, 16>(a, s);
    if (R == 32 && SG == 8) return launch_pk_shape<32, 8, 4>(a, s);
    return hipErrorInvalidValue;
}

}  // namespace swk
