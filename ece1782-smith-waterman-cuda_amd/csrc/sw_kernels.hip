// sw_kernels.hip — gfx950 (CDNA4) Smith-Waterman score-only kernels.
//
// Recurrence (the reference's, SWSolver.cu:246; cpu.cpp:43-74), linear gap g:
//     H(i,j) = max(0, H(i-1,j-1) + S[q_i][s_j], H(i,j-1) - g, H(i-1,j) - g)
// and its affine generalisation (Gotoh; go == ge reduces to the above):
//     E(i,j) = max(E(i,j-1) - ge, H(i,j-1) - go)
//     F(i,j) = max(F(i-1,j) - ge, H(i-1,j) - go)
//     H(i,j) = max(0, H(i-1,j-1) + S, E(i,j), F(i,j))
// score = max over all cells.  Integer max/add DP: no MFMA anywhere.
//
// Two kernels:
//  * inter   — one database subject per lane (the reference's parallelism,
//              SWSolver.cu:201-264, re-designed for wave64): the lane keeps R
//              query rows of its DP column in VGPRs, walks its subject left to
//              right, and hands the strip's bottom row to the next strip
//              through an int32 boundary row in HBM.  The query profile for
//              the strip (32 codes x R rows, int8) is staged in a wave-private
//              LDS slice; per column a lane reads its R scores with
//              ds_read_b128 at its own residue's row.  The per-cell sequence
//              is v_add_u32_sdwa (sign-extended profile byte) + v_max3_i32 +
//              v_sub_u32 clamp (+ half a v_max3 for the running maximum).
//  * intra   — one long subject per wave: lane t owns query rows
//              [t*RI, (t+1)*RI) of a 64*RI-row chunk and processes column
//              j = k - t at step k (anti-diagonal wavefront).  The bottom-row
//              H (and F) of lane t-1 and the residue code reach lane t through
//              DPP wave_shr:1; lane 0 is fed from the previous chunk's
//              boundary row, lane 63's output becomes the next chunk's.
//
// Profile bias: for the linear kernels the host stores S + g in the profile,
// so a cell is  h = usat(max3(H_left, H_up, H_diag + S + g) - g)  (the
// saturating subtract supplies the 0 floor; H_left, H_up >= 0).  For affine
// the profile holds S, and E/F are kept clamped at 0 (exact: a negative E or F
// can never win the max against the 0 floor, and clamping commutes with the
// "- ge" step because ge > 0).  The inter kernels carry E and F one cell
// AHEAD (Farrar's form): after H(i,j),  n = usat(H(i,j) - go),
// E(i,j+1) = max(usat(E(i,j) - ge), n),  F(i+1,j) = max(usat(F(i,j) - ge), n),
// so a cell is  h = max3(H_diag + S, E, F)  and n is shared by E and F; a
// strip's F boundary row therefore holds F of the next strip's first row.
#include "sw_int32.h"
#include "sw_kernels.h"

#include <cstdio>
#include <cstdlib>

namespace swk {

template <int R, int SG, bool AFFINE, bool SKEW>
__global__ __launch_bounds__(256) void sw_inter(InterArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kWavesPerWG * kProfileRows * inter_stride(R)];
    // threadIdx.x >> 6 is wave-uniform, but the compiler cannot prove it:
    // without readfirstlane every bound below would be a divergent VGPR value.
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    uint8_t* lp = lds + wave * (kProfileRows * inter_stride(R));
    if (a.blk_list) {  // rescue mode: the listed blocks only (count on the device)
        const int n = __builtin_amdgcn_readfirstlane(*a.blk_count);
        for (int i = blockIdx.x * kWavesPerWG + wave; i < n; i += gridDim.x * kWavesPerWG)
            inter_block<R, SG, AFFINE, SKEW>(a, list_take(a.blk_list, i), lp, lane);
        return;
    }
    const int blk = a.blk_first + blockIdx.x * kWavesPerWG + wave;
    if (blk >= a.nblocks) return;  // wave-uniform
    inter_block<R, SG, AFFINE, SKEW>(a, blk, lp, lane);
}

// ---------------------------------------------------------------------------
// inter-sequence, cooperative: one workgroup per WIDE block
// ---------------------------------------------------------------------------
// With one block per wave, the widest blocks (subjects near the long
// threshold) are the kernel's critical path: a 1536-column block is ~7 ms of
// one wave's work at 2 waves/SIMD.  Here the 4 waves of a workgroup share one
// block: in pass p wave w computes query strip 4p+w, one 8-column chunk behind
// wave w-1, and receives that wave's strip-bottom row (H, and F for affine)
// for the chunk through an LDS double buffer (one workgroup barrier per chunk
// step).  Only the last strip of a pass hands its bottom row to the next pass
// through HBM.  The block's latency drops ~4x.
template <int R, bool AFFINE, bool SKEW>
__global__ __launch_bounds__(256) void sw_inter_coop(InterArgs a) {
    constexpr int SG = 8;
    constexpr int S = inter_stride(R);
    constexpr int NF = AFFINE ? 2 : 1;  // rows handed down: H (+ F)
    __shared__ __attribute__((aligned(16))) uint8_t lds[kWavesPerWG * kProfileRows * S];
    __shared__ __attribute__((aligned(16))) int4 ring[NF][kWavesPerWG - 1][2][kLanes][SG / 4];
    __shared__ int red[kWavesPerWG][kLanes];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int blk = blockIdx.x;  // the widest blocks come first
    uint8_t* lp = lds + wave * (kProfileRows * S);
    const int nchunks = static_cast<int>(a.blk_groups[blk] * (kGroupCols / SG));
    const uint64_t base = a.blk_off[blk] + static_cast<uint64_t>(lane) * kGroupCols;
    const uint32_t go = static_cast<uint32_t>(a.gap_open);
    const uint32_t ge = static_cast<uint32_t>(a.gap_extend);
    const int nstrips = a.qpad / R;
    const int passes = (nstrips + kWavesPerWG - 1) / kWavesPerWG;
    int best = 0;

    for (int p = 0; p < passes; ++p) {
        const int strip = p * kWavesPerWG + wave;
        const bool valid = strip < nstrips;
        const bool first = (strip == 0);
        const bool last = (strip == nstrips - 1);
        const int s0 = strip * R;
        if (valid) stage_profile<R>(lp, a.prof, a.prof_stride, s0, lane);
        int H[R];
        int E[AFFINE ? R : 1];
#pragma unroll
        for (int r = 0; r < R; ++r) H[r] = 0;
#pragma unroll
        for (int r = 0; r < (AFFINE ? R : 1); ++r) E[r] = 0;
        int dtop = 0;
        __syncthreads();  // profile staged; the previous pass's HBM boundary rows are visible

        for (int t = 0; t < nchunks + kWavesPerWG - 1; ++t) {
            const int c = t - wave;
            if (valid && c >= 0 && c < nchunks) {
                const int col0 = c * SG;
                const uint64_t idx = base + (col0 >> 4) * kGroupBytes + (col0 & 15);
                Residues<SG> rs;
                rs.load(a.residues + idx);
                int bv[SG];
                int bf[AFFINE ? SG : 1];
                if (first) {
#pragma unroll
                    for (int q = 0; q < SG; ++q) bv[q] = 0;
#pragma unroll
                    for (int q = 0; q < (AFFINE ? SG : 1); ++q) bf[q] = 0;
                } else if (wave == 0) {
                    load_row<SG>(bv, a.bnd_h + idx);
                    if constexpr (AFFINE) load_row<SG>(bf, a.bnd_f + idx);
                } else {
#pragma unroll
                    for (int k = 0; k < NF; ++k) {
                        const int4* rp = ring[k][wave - 1][(t - 1) & 1][lane];
                        int* d = k == 0 ? bv : bf;
#pragma unroll
                        for (int q = 0; q < SG / 4; ++q) {
                            const int4 v = rp[q];
                            d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
                        }
                    }
                }
                int4 pa[R / 16], pb[R / 16];
                read_prof<R>(pa, lp, rs.code(0), 0);
                if constexpr (SKEW) read_prof<R>(pb, lp, rs.code(1), 0);
                sweep_group<R, SG, AFFINE, SKEW>(H, E, bv, bf, dtop, best, lp, rs, rs, false, pa, pb, go, ge);
                if (!last) {
                    if (wave == kWavesPerWG - 1) {
                        store_row<SG>(a.bnd_h + idx, bv);
                        if constexpr (AFFINE) store_row<SG>(a.bnd_f + idx, bf);
                    } else {
#pragma unroll
                        for (int k = 0; k < NF; ++k) {
                            int4* wp = ring[k][wave][t & 1][lane];
                            const int* d = k == 0 ? bv : bf;
#pragma unroll
                            for (int q = 0; q < SG / 4; ++q)
                                wp[q] = make_int4(d[4 * q], d[4 * q + 1], d[4 * q + 2], d[4 * q + 3]);
                        }
                    }
                }
            }
            __syncthreads();  // chunk step: ring slots written at t are read at t + 1
        }
    }
    red[wave][lane] = best;
    __syncthreads();
    if (wave == 0) {
        const int b = max(max(red[0][lane], red[1][lane]), max(red[2][lane], red[3][lane]));
        const int id = a.lane_ids[static_cast<size_t>(blk) * kLanes + lane];
        if (id >= 0) a.scores[id] = b;
    }
}

constexpr int kCoopRows = 32;
int inter_coop_rows() { return kCoopRows; }

hipError_t launch_inter_coop(const InterArgs& a, int ncoop, bool affine, bool sk, hipStream_t s) {
    if (ncoop <= 0 || a.qpad <= 0) return hipSuccess;
    const dim3 grid(ncoop), block(kWavesPerWG * kLanes);
    if (affine && sk) hipLaunchKernelGGL((sw_inter_coop<kCoopRows, true, true>), grid, block, 0, s, a);
    else if (affine) hipLaunchKernelGGL((sw_inter_coop<kCoopRows, true, false>), grid, block, 0, s, a);
    else if (sk) hipLaunchKernelGGL((sw_inter_coop<kCoopRows, false, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((sw_inter_coop<kCoopRows, false, false>), grid, block, 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// intra-sequence wavefront (one long subject per wave)
// ---------------------------------------------------------------------------
template <int RI, bool AFFINE>
__global__ __launch_bounds__(64) void sw_intra(IntraArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kProfileRows * intra_stride(RI)];
    if (a.list_count) {
        // list mode: re-scores the subjects a packed kernel flagged
        const int n = __builtin_amdgcn_readfirstlane(*a.list_count);
        for (int i = blockIdx.x; i < n; i += gridDim.x) intra_subject<RI, AFFINE>(a, list_take(a.subj_list, i), lds);
        return;
    }
    if (static_cast<int>(blockIdx.x) < a.nsubj) intra_subject<RI, AFFINE>(a, blockIdx.x, lds);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
// Inter-kernel shape (sw_kernels.h InterShape); o.inter_variant "RxSG"
// overrides (tuning only).
InterShape inter_shape(bool affine, int x2_ok, const sw_opts& o) {
    // measured on MI355X (scripts/tune_inter.py, profiles/r01_tune_inter*.jsonl,
    // r01_x2s/): int16-safe scans (the common case) run the packed two-strips-
    // per-lane kernel sw_inter_x2s, one subject per lane, in its fp16 form
    // (biased cell, v_pk_maximum3_f16; C2 affine 9.4 TCUPS vs 6.25 int16),
    // always guarded (rescue chain fp16 -> int16 -> int32).  Otherwise int32:
    // affine 32x8, linear 64x8 (+ the cooperative kernel for wide blocks).
    // Beyond the static int16 bound the packed kernel runs guarded (blocks
    // reaching kSat16 are re-scored at int32); o.int16_guard = 0 disables that.
    // (Measured slower and removed in round 2: 16-bit-value and int32-profile
    // one-subject kernels, pair-table packing, two subjects per lane, the
    // column-skewed int32 kernel; their numbers are in profiles/r01_tune_*.)
    const bool y_ok = x2_ok == 2 || (x2_ok == 1 && o.int16_guard != 0);
    InterShape v = y_ok ? InterShape{64, 8, true, true} : InterShape{affine ? 32 : 64, 8};
    // o.inter_variant (tests / A-B only): "RxSG" int32 (32x8, 64x8),
    // "y32x8" the int16 two-strips kernel, "f32x8" / "f32x4" its fp16 form
    if (const char* e = o.inter_variant; e[0]) {
        int r = 0, g = 0;
        if (std::sscanf(e, "f%dx%d", &r, &g) == 2 && y_ok && r == 32 && (g == 8 || (g == 4 && affine)))
            v = InterShape{2 * r, g, true, true};
        else if (std::sscanf(e, "y%dx%d", &r, &g) == 2 && y_ok && r == 32 && g == 8)
            v = InterShape{2 * r, g, true, false};  // R = rows per pass
        else if (std::sscanf(e, "%dx%d", &r, &g) == 2 && g == 8 && (r == 32 || r == 64))
            v = InterShape{r, g};
    }
    return v;
}

const char* inter_kernel_name(const InterShape& v, bool affine) {
    if (v.x2s) {
        static thread_local char b2[64];
        std::snprintf(b2, sizeof b2, "sw_inter_x2s<%d,%d,%s%s>", v.R / 2, v.SG, affine ? "affine" : "linear",
                      v.f16 ? ",fp16" : "");
        return b2;
    }
    static thread_local char buf[96];
    std::snprintf(buf, sizeof buf, "sw_inter<%d,%d,%s>", v.R, v.SG, affine ? "affine" : "linear");
    return buf;
}

// int32 re-scoring of the blocks a 16-bit kernel put on the rescue list.
int rescue_rows(bool affine) { return affine ? 32 : 64; }
hipError_t launch_inter_rescue(const InterArgs& a, bool affine, hipStream_t s) {
    // A few hundred waves walk the device-side list; an empty list costs one
    // tiny launch and no host synchronisation.
    if (affine)
        hipLaunchKernelGGL((sw_inter<32, 8, true, false>), dim3(64), dim3(kWavesPerWG * kLanes), 0, s, a);
    else
        hipLaunchKernelGGL((sw_inter<64, 8, false, false>), dim3(64), dim3(kWavesPerWG * kLanes), 0, s, a);
    return hipGetLastError();
}

// Rows per lane for the intra kernel: minimise
//   chunks * (steps per chunk) * (ops per step)
// with ops per step ~ RI * 3.7 (cells) + 8 (hand-off overhead); RI is even
// and at most 16 (register budget).
int intra_rows_for(int qlen, int longest) {
    int best_ri = 16;
    double best_cost = 1e300;
    for (int ri = 2; ri <= 16; ri += 2) {
        const int chunk = kLanes * ri;
        const int nch = (qlen + chunk - 1) / chunk;
        const double cost = static_cast<double>(nch) * (longest + kLanes - 1) * (ri * 3.7 + 8.0);
        if (cost < best_cost) { best_cost = cost; best_ri = ri; }
    }
    return best_ri;
}

int intra_chunk_bytes(int ri) { return kProfileRows * kLanes * intra_rip(ri); }

hipError_t launch_inter(const InterArgs& a, bool affine, const InterShape& v, hipStream_t s) {
    if (a.nblocks - a.blk_first <= 0 || a.qpad <= 0) return hipSuccess;
    const dim3 grid((a.nblocks - a.blk_first + kWavesPerWG - 1) / kWavesPerWG);
    const dim3 block(kWavesPerWG * kLanes);
    if (v.x2s) return launch_inter_x2s(a, v.R / 2, v.SG, affine, v.f16, s);
#define SW_LAUNCH_INTER(R_, SG_)                                                                         \
    if (v.R == R_ && v.SG == SG_) {                                                                      \
        if (affine) hipLaunchKernelGGL((sw_inter<R_, SG_, true, false>), grid, block, 0, s, a);          \
        else hipLaunchKernelGGL((sw_inter<R_, SG_, false, false>), grid, block, 0, s, a);                \
        return hipGetLastError();                                                                        \
    }
    SW_LAUNCH_INTER(32, 8)
    SW_LAUNCH_INTER(64, 8)
#undef SW_LAUNCH_INTER
    return hipErrorInvalidValue;
}

template <int RI>
static void launch_intra_ri(const IntraArgs& a, bool affine, hipStream_t s) {
    // list mode: one workgroup per possible entry (surplus ones return at
    // once), so a long list runs as wide as a full scan
    const dim3 grid(a.nsubj);
    if (affine)
        hipLaunchKernelGGL((sw_intra<RI, true>), grid, dim3(kLanes), 0, s, a);
    else
        hipLaunchKernelGGL((sw_intra<RI, false>), grid, dim3(kLanes), 0, s, a);
}

hipError_t launch_intra(const IntraArgs& a, int ri, bool affine, hipStream_t s) {
    if (a.nsubj <= 0 || a.qpad <= 0) return hipSuccess;
    switch (ri) {
        case 2: launch_intra_ri<2>(a, affine, s); break;
        case 4: launch_intra_ri<4>(a, affine, s); break;
        case 6: launch_intra_ri<6>(a, affine, s); break;
        case 8: launch_intra_ri<8>(a, affine, s); break;
        case 10: launch_intra_ri<10>(a, affine, s); break;
        case 12: launch_intra_ri<12>(a, affine, s); break;
        case 14: launch_intra_ri<14>(a, affine, s); break;
        case 16: launch_intra_ri<16>(a, affine, s); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace swk
