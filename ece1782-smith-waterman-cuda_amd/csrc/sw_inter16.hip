// sw_inter16.hip — inter-sequence Smith-Waterman with 16-bit cell values.
//
// Same blocking as sw_inter (sw_kernels.hip): one wave = 64 subjects, one per
// lane; R query rows per strip in VGPRs; profile slice in wave-private LDS;
// strip boundary rows in HBM (here as u16, half the traffic).
//
// Why 16-bit: on gfx950 the VOP2 16-bit ops (v_add_u16, v_max_i16/u16,
// v_sub_u16 clamp) dual-issue across waves (~2.4-3 cycles per wave64
// instruction), while every 32-bit max/max3, SDWA and packed op costs ~4.2
// (profiles/r01_valu_rate_*.txt).  A 5-op 16-bit cell measured 12.0-13.1
// cycles against 15.9-18.2 for the int32 cell.
//
// This translation unit is built with -mllvm -amdgpu-sdwa-peephole=0, and the
// two maxima of a cell alternate unsigned/signed forms, so that hipcc does not
// fuse them into v_max3_i16 (8.3 cycles) or SDWA adds (4.2).  H values stay in
// 0..32767 (profile values are gap-biased scores); a lane whose running
// maximum reaches kSat16 may have overflowed, and its block is appended to a
// rescue list that the int32 kernel re-scores.
#include "sw_kernels.h"

namespace swk {

typedef uint16_t u16;
typedef int16_t i16;

__device__ __forceinline__ u16 umx(u16 a, u16 b) { return a > b ? a : b; }
__device__ __forceinline__ u16 smx(u16 a, u16 b) {
    return static_cast<u16>(static_cast<i16>(a) > static_cast<i16>(b) ? a : b);
}
__device__ __forceinline__ u16 usat(u16 a, u16 g) { return __builtin_elementwise_sub_sat(a, g); }

__host__ __device__ constexpr int inter16_stride(int R) {
    // 2R bytes + 16, with an odd number of 16-byte slots (bank spread)
    return ((2 * R + 16) / 16) % 2 == 1 ? 2 * R + 16 : 2 * R + 32;
}

template <int R>
__device__ __forceinline__ void stage_profile16(uint8_t* lp, const int16_t* __restrict__ prof, int stride, int s0,
                                                int lane) {
    constexpr int kChunks = kProfileRows * (R / 8);  // 16-byte chunks = 8 rows
    constexpr int S = inter16_stride(R);
#pragma unroll
    for (int t = lane; t < kChunks; t += kLanes) {
        const int c = t / (R / 8);
        const int k = t % (R / 8);
        const int4 v = *reinterpret_cast<const int4*>(prof + static_cast<size_t>(c) * stride + s0 + 8 * k);
        *reinterpret_cast<int4*>(lp + c * S + 16 * k) = v;
    }
}

// `dep` ties the read to a value of the previous chunk so the scheduler
// cannot hoist every unrolled read to the top of the body.
__device__ __forceinline__ void read_chunk16(int4 (&p)[2], const uint8_t* lp, uint32_t off, uint32_t dep) {
    asm volatile("" : "+v"(off) : "v"(dep));
    const int4* pp = reinterpret_cast<const int4*>(lp + off);
    p[0] = pp[0];
    p[1] = pp[1];
}

template <int R, int SG>
__global__ __launch_bounds__(256) void sw_inter16(InterArgs a) {
    static_assert(SG % 8 == 0, "boundary rows move as 16-byte groups of 8 u16");
    constexpr int S = inter16_stride(R);
    constexpr int NCH = R / 16;  // 16-row chunks (2 x ds_read_b128)
    constexpr int STEPS = SG * NCH;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kWavesPerWG * kProfileRows * S];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int blk = blockIdx.x * kWavesPerWG + wave;
    if (blk >= a.nblocks) return;
    uint8_t* lp = lds + wave * (kProfileRows * S);
    const int16_t* prof16 = reinterpret_cast<const int16_t*>(a.prof);
    uint16_t* bnd16 = reinterpret_cast<uint16_t*>(a.bnd_h);

    const uint32_t ncols = a.blk_groups[blk] * kGroupCols;
    const uint64_t base = a.blk_off[blk] + static_cast<uint64_t>(lane) * kGroupCols;
    const u16 go = static_cast<u16>(a.gap_open);
    u16 best = 0;
    if (ncols == 0) goto done;

    for (int s0 = 0; s0 < a.qpad; s0 += R) {
        const bool first = (s0 == 0);
        const bool last = (s0 + R >= a.qpad);
        stage_profile16<R>(lp, prof16, a.prof_stride, s0, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");

        u16 H[R];
#pragma unroll
        for (int r = 0; r < R; ++r) H[r] = 0;
        u16 dtop = 0;

        Residues<SG> rs, rs_next;
        uint32_t bw[SG / 2], bw_next[SG / 2];  // boundary row: u16 pairs
        rs.load(a.residues + base);
        if (!first) {
#pragma unroll
            for (int q = 0; q < SG / 8; ++q) {
                const int4 v = *reinterpret_cast<const int4*>(bnd16 + base + 8 * q);
                bw[4 * q] = v.x; bw[4 * q + 1] = v.y; bw[4 * q + 2] = v.z; bw[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int q = 0; q < SG / 2; ++q) bw[q] = 0;
        }
        int4 P[2][2];
        read_chunk16(P[0], lp, rs.code(0) * S, 0);

        for (uint32_t col0 = 0; col0 < ncols; col0 += SG) {
            const uint64_t idx = base + (col0 >> 4) * kGroupBytes + (col0 & 15);
            const bool more = col0 + SG < ncols;
            const uint64_t nidx = base + ((col0 + SG) >> 4) * kGroupBytes + ((col0 + SG) & 15);
            if (more) {
                rs_next.load(a.residues + nidx);
                if (!first) {
#pragma unroll
                    for (int q = 0; q < SG / 8; ++q) {
                        const int4 v = *reinterpret_cast<const int4*>(bnd16 + nidx + 8 * q);
                        bw_next[4 * q] = v.x; bw_next[4 * q + 1] = v.y;
                        bw_next[4 * q + 2] = v.z; bw_next[4 * q + 3] = v.w;
                    }
                }
            }
            u16 out[SG];
            u16 up = 0, diag = 0;
#pragma unroll
            for (int t = 0; t < STEPS; ++t) {
                const int jj = t / NCH;
                const int k = t % NCH;
                if (t + 1 < STEPS) {
                    const int jn = (t + 1) / NCH, kn = (t + 1) % NCH;
                    read_chunk16(P[(t + 1) & 1], lp, rs.code(jn) * S + 32 * kn, k == 0 ? H[R - 1] : H[16 * k - 1]);
                } else if (more) {
                    read_chunk16(P[(t + 1) & 1], lp, rs_next.code(0) * S, H[16 * k - 1]);
                }
                if (k == 0) {
                    up = static_cast<u16>((jj & 1) ? (bw[jj >> 1] >> 16) : bw[jj >> 1]);
                    diag = dtop;
                    dtop = up;
                }
                const int4(&pc)[2] = P[t & 1];
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const uint32_t pw[4] = {static_cast<uint32_t>(pc[q].x), static_cast<uint32_t>(pc[q].y),
                                            static_cast<uint32_t>(pc[q].z), static_cast<uint32_t>(pc[q].w)};
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const int r = 16 * k + 8 * q + e;
                        const u16 sc = static_cast<u16>((e & 1) ? (pw[e >> 1] >> 16) : pw[e >> 1]);
                        const u16 m = smx(umx(H[r], up), static_cast<u16>(diag + sc));
                        const u16 h = usat(m, go);
                        diag = H[r];
                        H[r] = h;
                        up = h;
                        best = (r & 1) ? smx(best, h) : umx(best, h);
                    }
                }
                if (k == NCH - 1) {
                    out[jj] = up;
                    asm volatile("" : "+v"(best));
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            if (!last) {
#pragma unroll
                for (int q = 0; q < SG / 8; ++q)
                    *reinterpret_cast<int4*>(bnd16 + idx + 8 * q) =
                        make_int4(static_cast<int>(out[8 * q] | (static_cast<uint32_t>(out[8 * q + 1]) << 16)),
                                  static_cast<int>(out[8 * q + 2] | (static_cast<uint32_t>(out[8 * q + 3]) << 16)),
                                  static_cast<int>(out[8 * q + 4] | (static_cast<uint32_t>(out[8 * q + 5]) << 16)),
                                  static_cast<int>(out[8 * q + 6] | (static_cast<uint32_t>(out[8 * q + 7]) << 16)));
            }
            if (more) {
                rs = rs_next;
#pragma unroll
                for (int q = 0; q < SG / 2; ++q) bw[q] = first ? 0u : bw_next[q];
            }
        }
    }
done:
    {
        const int b16 = static_cast<int>(static_cast<i16>(best));
        const bool saturated = b16 >= kSat16 || b16 < 0;
        const int id = a.lane_ids[static_cast<size_t>(blk) * kLanes + lane];
        if (id >= 0) a.scores[id] = b16 < 0 ? 0 : b16;
        if (__builtin_amdgcn_ballot_w64(saturated) != 0 && lane == 0) {
            const int slot = atomicAdd(a.rescue_count, 1);
            a.rescue_list[slot] = blk;
        }
    }
}

hipError_t launch_inter16(const InterArgs& a, int R, int SG, hipStream_t s) {
    if (a.nblocks <= 0 || a.qpad <= 0) return hipSuccess;
    const dim3 grid((a.nblocks + kWavesPerWG - 1) / kWavesPerWG);
    const dim3 block(kWavesPerWG * kLanes);
#define SW_LAUNCH_I16(R_, SG_)                                                       \
    if (R == R_ && SG == SG_) {                                                      \
        hipLaunchKernelGGL((sw_inter16<R_, SG_>), grid, block, 0, s, a);             \
        return hipGetLastError();                                                    \
    }
    SW_LAUNCH_I16(64, 8)
    SW_LAUNCH_I16(64, 16)
    SW_LAUNCH_I16(32, 8)
    SW_LAUNCH_I16(32, 16)
    SW_LAUNCH_I16(48, 8)
#undef SW_LAUNCH_I16
    return hipErrorInvalidValue;
}

}  // namespace swk
