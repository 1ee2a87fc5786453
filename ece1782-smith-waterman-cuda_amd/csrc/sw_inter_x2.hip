// sw_inter_x2.hip — inter-sequence Smith-Waterman in packed 16-bit cells
// (the reference's f_scoreSequenceTiledCoalesced,
// SWSolver.cu:201-264): sw_inter_x2s (one subject per lane, TWO query strips
// per pass, one wave per 64-subject block), its wave-group form sw_inter_x2p
// (a block's passes split over 2 or 4 waves) and sw_scan_lpt (the whole scan
// of a small database, inter blocks and long subjects, in one longest-first
// launch that also re-scores what it flags).
//
// Why: the scan is bound by VALU issue.  On gfx950 every 32-bit max/max3 and
// the SDWA byte add issue at the slow ~4.3-cycle rate, so an int32 affine cell
// costs ~26 SIMD-cycles per 64 cells (profiles/r01_valu_rate_*.txt); one
// v_pk_* instruction (also ~4.25 cycles) updates TWO cells.
//
// The default cell is fp16 with a bias (x2s_pass): cell (r, jj)
// of an 8-column sub-group stores H + (r % 16 + jj) ge, so both gap
// extensions are the drift of the bias and an affine cell pair is 5 packed
// ops (v_pk_fma_f16 for H_diag + S, v_pk_maximum3_f16 for H, v_pk_add_f16
// for H - (go - ge), a max for E, a max3 for F with the floor), a linear one
// 3; the running maxima are kept per anti-diagonal.  The lane's low halves run
// rows [s0, s0 + 32) at column t, the high halves rows [s0 + 32, s0 + 64) at
// column t - 8, fed through an 8-entry register delay line, so a 64-row pass
// hands one dword (H | F << 16) per column to the next pass through HBM.
// The pair (S_low, S_high) is formed without a combine: the LDS images hold
// (S, 1) and (1, S) and the fma multiplies them.
//
// Exactness: every fp16 value carries the offset -2048 + 2 ge, so true scores
// up to ~4,000 are exact integers; a lane whose maximum reaches the guard band
// (a.sat_limit) flags its block, which the int16 form of the same kernel
// re-scores (x2s_block with F16 = false: up to 32767, guard kSat16), and
// blocks it flags again go to the int32 kernel (sw_int32.h).  Blocks and
// subjects are listed on the device (sw_kernels.h list_publish / list_take);
// no host synchronisation anywhere in the chain.
#include <algorithm>

#include "sw_int32.h"
#include "sw_intra_x2.h"
#include "sw_kernels.h"

namespace swk {

typedef short s2 __attribute__((ext_vector_type(2)));
typedef unsigned short u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ s2 as_s2(uint32_t x) { return __builtin_bit_cast(s2, x); }
__device__ __forceinline__ uint32_t as_u32(s2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ s2 max2(s2 a, s2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ s2 usub2(s2 a, u2 g) {
    return __builtin_bit_cast(s2, __builtin_elementwise_sub_sat(__builtin_bit_cast(u2, a), g));
}

// dwords per code row of an LDS image: R, padded to an odd number of
// 16-byte slots so lanes reading different codes spread over the banks
__host__ __device__ constexpr int x2_row_dwords(int R) { return (R / 4) % 2 == 1 ? R : R + 4; }

// Profile codes an image holds: the 25 residue codes and the pad code (the
// database holds no others; sw_db_create validates every byte).
constexpr int kImgCodes = kPadCode + 1;

// One wave's profile images: `lo` / `hi` for the two strips of a pass.
// (Copies for column 0 of every sub-group, one sub-group's bias lower, would
// save the per-sub-group rebase of H: 2 % fewer VALU instructions on C2, but
// at 77 KB of LDS per pair workgroup the scan ran 2 % SLOWER beside the
// long-subject kernel, 7.43 against 7.25 ms per step; not kept.)
template <int R>
struct __attribute__((aligned(16))) X2Lds {  // 16-byte aligned: the waves' images are read by ds_read_b128
    static constexpr int kImg = kImgCodes * x2_row_dwords(R);
    uint32_t lo[kImg];
    uint32_t hi[kImg];
};
static_assert(sizeof(X2Lds<32>) % 16 == 0 && sizeof(X2Lds<48>) % 16 == 0, "image alignment");

template <int N>
__device__ __forceinline__ uint32_t word(const int4 (&v)[N], int w) {
    const int4 q = v[w >> 2];
    switch (w & 3) {
        case 0: return static_cast<uint32_t>(q.x);
        case 1: return static_cast<uint32_t>(q.y);
        case 2: return static_cast<uint32_t>(q.z);
        default: return static_cast<uint32_t>(q.w);
    }
}

template <int SG>
__device__ __forceinline__ void load_codes(uint32_t (&w)[SG / 4], const uint8_t* p, bool valid) {
    if (valid) {
        if constexpr (SG == 16) {
            const int4 v = *reinterpret_cast<const int4*>(p);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        } else if constexpr (SG == 8) {
            const int2 v = *reinterpret_cast<const int2*>(p);
            w[0] = v.x; w[1] = v.y;
        } else {
            w[0] = *reinterpret_cast<const uint32_t*>(p);
        }
    } else {
#pragma unroll
        for (int q = 0; q < SG / 4; ++q) w[q] = 0x19191919u;  // kPadCode in every byte
    }
}

__device__ __forceinline__ uint32_t code_of(const uint32_t* w, int jj) { return (w[jj >> 2] >> (8 * (jj & 3))) & 0xffu; }

// LDS byte address base + code(jj) * RB of column jj's profile row in ONE
// v_dot4_u32_u8 (byte jj & 3 of the code word times RB in the same byte of
// the constant) instead of a byte extract and a multiply-add
template <uint32_t RB>
__device__ __forceinline__ uint32_t code_row(const uint32_t* w, int jj, uint32_t base) {
    static_assert(RB < 256, "row stride must fit a byte");
    return __builtin_amdgcn_udot4(w[jj >> 2], RB << (8 * (jj & 3)), base, false);
}

template <int SG>
__device__ __forceinline__ void load_pairs(uint32_t (&v)[SG], const int32_t* p) {
#pragma unroll
    for (int q = 0; q < SG / 4; ++q) {
        const int4 t = *reinterpret_cast<const int4*>(p + 4 * q);
        v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
    }
}

template <int SG>
__device__ __forceinline__ void store_pairs(int32_t* p, const uint32_t (&v)[SG]) {
#pragma unroll
    for (int q = 0; q < SG / 4; ++q)
        *reinterpret_cast<int4*>(p + 4 * q) = make_int4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}

// half-word shuffles as one v_perm_b32 each (byte i of the result = byte
// sel[i] of {src0 : src1}, src1 the low dword): (a.lo, b.lo), (a.hi, b.lo),
// (a.hi, b.hi)
__device__ __forceinline__ uint32_t lo_lo(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x05040100u); }
__device__ __forceinline__ uint32_t hi_lo(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x05040302u); }
__device__ __forceinline__ uint32_t hi_hi(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); }

// The pass hand-off in HBM, SG columns from index i of the residues' index
// space: affine (H | F << 16) dwords; linear H alone as 16-bit values (with
// open = extend the biased cell needs no F: half the bytes).  Per column
// the value lands in v[q] with H in its low half (even q) or its high half
// (odd q; col_start picks the matching half).
template <int SG, bool AFFINE>
__device__ __forceinline__ void load_bnd(uint32_t (&v)[SG], const uint32_t* bnd, uint64_t i) {
    if constexpr (AFFINE) {
        load_pairs<SG>(v, reinterpret_cast<const int32_t*>(bnd) + i);
    } else {
        const uint16_t* p = reinterpret_cast<const uint16_t*>(bnd) + i;
        uint32_t w[SG / 2];
        if constexpr (SG == 8) {
            const int4 t = *reinterpret_cast<const int4*>(p);
            w[0] = t.x; w[1] = t.y; w[2] = t.z; w[3] = t.w;
        } else {
            static_assert(SG == 4, "sub-group width");
            const int2 t = *reinterpret_cast<const int2*>(p);
            w[0] = t.x; w[1] = t.y;
        }
#pragma unroll
        for (int q = 0; q < SG; ++q) v[q] = w[q / 2];
    }
}
// hb[q]: affine (H | F << 16) of column q; linear H of column q in BOTH halves
template <int SG, bool AFFINE>
__device__ __forceinline__ void store_bnd(uint32_t* bnd, uint64_t i, const uint32_t (&hb)[SG]) {
    if constexpr (AFFINE) {
        store_pairs<SG>(reinterpret_cast<int32_t*>(bnd) + i, hb);
    } else {
        uint16_t* p = reinterpret_cast<uint16_t*>(bnd) + i;
        uint32_t w[SG / 2];
#pragma unroll
        for (int q = 0; q < SG / 2; ++q) w[q] = lo_lo(hb[2 * q], hb[2 * q + 1]);
        if constexpr (SG == 8) *reinterpret_cast<int4*>(p) = make_int4(w[0], w[1], w[2], w[3]);
        else *reinterpret_cast<int2*>(p) = make_int2(w[0], w[1]);
    }
}

// ---------------------------------------------------------------------------
// sw_inter_x2s: ONE subject per lane, TWO query strips per pass
// ---------------------------------------------------------------------------
// The low 16 bits of a lane's registers run rows [s0, s0+R) of its subject at
// column t while the high 16 bits run rows [s0+R, s0+2R) of the same subject
// at column t-SG.  The low strip's bottom row (H, F) reaches the high strip
// SG steps later through an SG-entry register delay line (the values a
// sub-group of SG columns produces are consumed by the next sub-group at the
// same position), so only every second strip boundary goes through HBM, as
// one dword (H | F << 16) per packed column per lane: 4x less boundary
// traffic than sw_inter_x2 (2 dwords per 2 subjects per R rows), and 64
// subjects per wave (finer work units, shorter tail).  Cost: the first
// sub-group of a pass computes the high strip on SG virtual columns before
// the subject (all-zero inputs, pad scores: they stay 0) and the last one the
// low strip on SG pad columns after it.  Same packed cell as sw_inter_x2; the
// score pair is lo[code(t)][i] | hi[code(t-SG)][i] with the two images holding
// the two strips' rows.
// F16: the images hold the scores as fp16 bit patterns (exact integers).
__device__ __forceinline__ uint32_t to_f16_bits(uint32_t v16) {
    return static_cast<uint32_t>(__builtin_bit_cast(uint16_t, static_cast<_Float16>(static_cast<int16_t>(v16))));
}

// Stage the profile images of one pass: img 0 (lo) <- rows [s0, s0+R), img 1
// (hi) <- rows [s0+R, s0+2R), both when img < 0 (2 x 26 codes x R/8 int4
// loads of 8 rows each, spread over the lanes).  Each dword pairs a row's
// score with 1 (1.0 in fp16) in the other half: the kernel forms the pair
// as lo * hi + H_diag in one v_pk_fma_f16 / v_pk_mad_u16.
// F16: the images hold S + bias (the column-biased cell's gap extension), and
// the first row of each 16-row group S + bias + bias0: the diagonal entering
// that row still carries the previous row group's bias, 16 ge above its own
// (bias0 = -16 ge folds the shift back into the profile; see x2s_pass).
template <int R, bool F16>
__device__ __forceinline__ void stage_x2s(X2Lds<R>& L, const int16_t* __restrict__ prof, int stride, int s0,
                                          int lane, int bias, int bias0, int img) {
    constexpr int RD = x2_row_dwords(R);
    constexpr int PER = kImgCodes * (R / 8);  // int4 loads per image
    constexpr uint32_t one = F16 ? 0x3c00u : 1u;
    const int n = img < 0 ? 2 * PER : PER;
    for (int t = lane; t < n; t += kLanes) {
        const int im = img < 0 ? t / PER : img;
        const int u = img < 0 ? t % PER : t;
        const int c = u / (R / 8);
        const int k = u % (R / 8);
        const int4 v = *reinterpret_cast<const int4*>(prof + static_cast<size_t>(c) * stride + s0 + im * R + 8 * k);
        const uint32_t w[4] = {static_cast<uint32_t>(v.x), static_cast<uint32_t>(v.y), static_cast<uint32_t>(v.z),
                               static_cast<uint32_t>(v.w)};
        uint32_t o[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int s0v = static_cast<int16_t>(w[e] & 0xffffu), s1v = static_cast<int16_t>(w[e] >> 16);
            // row 8k + 2e of the strip starts a row group when k is even and e = 0
            const int b0 = (F16 && k % 2 == 0 && e == 0) ? bias0 : 0;
            uint32_t a0 = static_cast<uint32_t>(s0v) & 0xffffu, a1 = static_cast<uint32_t>(s1v) & 0xffffu;
            if constexpr (F16) {
                a0 = to_f16_bits(static_cast<uint32_t>(s0v + bias + b0));
                a1 = to_f16_bits(static_cast<uint32_t>(s1v + bias));
            }
            o[2 * e] = im ? (a0 << 16) | one : a0 | (one << 16);
            o[2 * e + 1] = im ? (a1 << 16) | one : a1 | (one << 16);
        }
        int4* d = reinterpret_cast<int4*>((im ? L.hi : L.lo) + c * RD + 8 * k);
        d[0] = make_int4(o[0], o[1], o[2], o[3]);
        d[1] = make_int4(o[4], o[5], o[6], o[7]);
    }
}


typedef int v4i __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const v4i lds_int4;

// LDS byte address of a __shared__ object (the low half of its generic address)
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p));
}

// read_x2 for the two-strips images from precomputed LDS byte addresses of
// the two code rows (one v_mad each per column): the per-step tie to `dep`
// keeps the reads from being hoisted, and the chunk offset folds into the
// ds_read_b128 offset field.
template <int N>
__device__ __forceinline__ void read_x2a(int4 (&pl)[N], int4 (&ph)[N], uint32_t& aa, uint32_t& ab, int k,
                                         uint32_t dep) {
    asm volatile("" : "+v"(aa), "+v"(ab) : "v"(dep));
    lds_int4* a = reinterpret_cast<lds_int4*>(static_cast<uintptr_t>(aa)) + N * k;
    lds_int4* b = reinterpret_cast<lds_int4*>(static_cast<uintptr_t>(ab)) + N * k;
#pragma unroll
    for (int q = 0; q < N; ++q) {
        pl[q] = __builtin_bit_cast(int4, a[q]);
        ph[q] = __builtin_bit_cast(int4, b[q]);
    }
}

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

// The packed cell in two number formats.  int16: wrapping add, saturating
// subtract, v_pk_max_i16.  fp16 (affine only): v_pk_add_f16 and the gfx950
// three-input v_pk_maximum3_f16, which folds the 0 floor into E and F
// (E = max3(E - ge, n, 0)) and H's two maxima into one: 7.5 packed ops per
// cell pair instead of 9.66 (profiles/r01_f16_rate.txt).  fp16 holds every
// integer up to 2048 exactly.
template <bool F16>
struct PkCell;

template <>
struct PkCell<false> {
    using V = s2;
    static __device__ __forceinline__ V from(uint32_t x) { return as_s2(x); }
    static __device__ __forceinline__ uint32_t bits(V x) { return as_u32(x); }
};

template <>
struct PkCell<true> {
    using V = h2;
    static __device__ __forceinline__ V from(uint32_t x) { return __builtin_bit_cast(h2, x); }
    static __device__ __forceinline__ uint32_t bits(V x) { return __builtin_bit_cast(uint32_t, x); }
};

__device__ __forceinline__ h2 max3h(h2 a, h2 b, h2 c) {
    return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}

template <int R, int SG, bool AFFINE, bool F16, int CR = 16>
__device__ __forceinline__ bool x2s_block(const InterArgs& a, int blk, X2Lds<R>& L, int lane);

// LIST: a rescue stage walking the device-side block list (a separate
// instantiation, so the list loop costs the scan kernels no registers).
template <int R, int SG, bool AFFINE, bool F16, bool LIST, int CR = 16>
__global__ __launch_bounds__(256, 2) void sw_inter_x2s(InterArgs a) {
    static_assert(R % CR == 0 && SG % 4 == 0, "shape");
    __shared__ __attribute__((aligned(16))) X2Lds<R> lds[kWavesPerWG];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    X2Lds<R>& L = lds[wave];
    if constexpr (LIST) {
        const int n = __builtin_amdgcn_readfirstlane(*a.blk_count);
        for (int i = blockIdx.x * kWavesPerWG + wave; i < n; i += gridDim.x * kWavesPerWG)
            x2s_block<R, SG, AFFINE, F16, CR>(a, list_take(a.blk_list, i), L, lane);
        return;
    }
    const int blk = a.blk_first + blockIdx.x * kWavesPerWG + wave;
    if (blk >= a.nblocks) return;  // wave-uniform; waves never synchronise
    x2s_block<R, SG, AFFINE, F16, CR>(a, blk, L, lane);
}

// The fp16 cell's running maximum.  Cell (r, jj) of a sub-group (r = row of
// the strip, jj = column of the sub-group) holds H + (r % kRowGroup + jj) ge
// (see x2s_pass), so the maximum is kept per anti-diagonal k = r % 16 + jj:
// acc[k] gathers the cells of bias k ge, two per v_pk_maximum3_f16 (cell (r,
// jj) of an odd column with cell (r + 1, jj - 1), still in H[r + 1]).
constexpr int kRowGroup = 16;
constexpr int kAcc = kRowGroup + 8 - 1;
template <bool F16>
struct Best {
    typename PkCell<F16>::V v;
    __device__ __forceinline__ void init(const InterArgs&) { v = PkCell<F16>::from(0u); }
    __device__ __forceinline__ typename PkCell<F16>::V value(const InterArgs&) const { return v; }
};
template <>
struct Best<true> {
    h2 acc[kAcc];
    // the maxima start at the offset zero (every cell is at least that)
    __device__ __forceinline__ void init(const InterArgs& a) {
#pragma unroll
        for (int k = 0; k < kAcc; ++k) acc[k] = __builtin_bit_cast(h2, a.f16_zero);
    }
    __device__ __forceinline__ void pin() {
        static_assert(kAcc == 23, "pin list");
        asm volatile("" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]),
                     "+v"(acc[6]), "+v"(acc[7]));
        asm volatile("" : "+v"(acc[8]), "+v"(acc[9]), "+v"(acc[10]), "+v"(acc[11]), "+v"(acc[12]), "+v"(acc[13]),
                     "+v"(acc[14]), "+v"(acc[15]));
        asm volatile("" : "+v"(acc[16]), "+v"(acc[17]), "+v"(acc[18]), "+v"(acc[19]), "+v"(acc[20]),
                     "+v"(acc[21]), "+v"(acc[22]));
    }
    // the maximum with the bias removed but the offset kept (the true score
    // may exceed 2048, which fp16 no longer holds exactly; x2s_finish
    // removes the offset in integers)
    __device__ __forceinline__ h2 value(const InterArgs& a) const {
        const h2 z = __builtin_bit_cast(h2, a.f16_step[0]);
        h2 b = acc[0];
#pragma unroll
        for (int k = 1; k < kAcc; ++k)
            b = __builtin_elementwise_maximum(b, acc[k] - (__builtin_bit_cast(h2, a.f16_step[k]) - z));
        return b;
    }
};

// Block timeline for tail analysis (-DSW_TRACE_BLOCKS builds only).
__device__ __forceinline__ uint64_t trace_now() {
#ifdef SW_TRACE_BLOCKS
    return __builtin_amdgcn_s_memrealtime();
#else
    return 0;
#endif
}
__device__ __forceinline__ void trace_block(const InterArgs& a, int blk, uint64_t t0, int lane, uint32_t kind) {
#ifdef SW_TRACE_BLOCKS
    if (a.trace && lane == 0) {
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        const uint32_t hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11));  // HW_REG_XCC_ID
        uint64_t* t = a.trace + 4 * static_cast<size_t>(blk);
        t[0] = t0;
        t[1] = t1;
        t[2] = hw;
        t[3] = xcc | (static_cast<uint64_t>(kind) << 32);
    }
#else
    (void)a; (void)blk; (void)t0; (void)lane; (void)kind;
#endif
}

// Score and guard of one block (lane = subject).
// Guarded mode: H grows by at most max S per cell, so a lane whose values
// could have left the exact range has its running maximum in the guard
// band first — int16: [kSat16, 32767] (or wrapped: negative); fp16:
// >= a.sat_limit = 2048 - 2 max S, computed exactly — and its block is
// re-scored from the list by the next stage (int16 packed, then int32).
// Returns (wave-uniform) whether the block was appended to the rescue list.
template <bool F16>
__device__ __forceinline__ bool x2s_finish(const InterArgs& a, int blk, int lane, typename PkCell<F16>::V best) {
    int b;
    if constexpr (F16)  // offset removed in integers: true scores go up to ~4096
        b = static_cast<int>(static_cast<float>(__builtin_elementwise_maximum(best.x, best.y))) -
            static_cast<int>(static_cast<float>(__builtin_bit_cast(h2, a.f16_step[0]).x));
    else
        b = max(static_cast<int>(best.x), static_cast<int>(best.y));
    const int id = a.lane_ids[static_cast<size_t>(blk) * kLanes + lane];
    if (id >= 0) a.scores[id] = b;
    if (a.rescue_list) {
        const bool sat = F16 ? (b >= a.sat_limit) : (b >= kSat16 || b < 0);
        const uint64_t m = __builtin_amdgcn_ballot_w64(sat);
        if (m && lane == 0) {
            list_publish(a.rescue_list, a.rescue_count, blk);
            if (a.rescue_max) atomicMax(a.rescue_max, blk);
        }
        return m != 0;
    }
    return false;
}


// LDS ring between the two waves of a pair (sw_inter_x2p): kRingSlots
// sub-groups of boundary dwords, lane-contiguous int4s (conflict-free b128).
constexpr int kRingSlots = 4;

template <int SG>
__device__ __forceinline__ void ring_store(int4* ring, int slot, int lane, const uint32_t (&v)[SG]) {
#pragma unroll
    for (int q = 0; q < SG / 4; ++q)
        ring[(slot * (SG / 4) + q) * kLanes + lane] = make_int4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}

template <int SG>
__device__ __forceinline__ void ring_load(uint32_t (&v)[SG], const int4* ring, int slot, int lane) {
#pragma unroll
    for (int q = 0; q < SG / 4; ++q) {
        const int4 t = ring[(slot * (SG / 4) + q) * kLanes + lane];
        v[4 * q] = static_cast<uint32_t>(t.x);
        v[4 * q + 1] = static_cast<uint32_t>(t.y);
        v[4 * q + 2] = static_cast<uint32_t>(t.z);
        v[4 * q + 3] = static_cast<uint32_t>(t.w);
    }
}

// Flag-synchronised wave groups (affine gaps): instead of one workgroup
// barrier per sub-group (a tick shared by every wave of the workgroup, the
// two pairs of a workgroup included), each wave publishes in LDS how many
// sub-groups it has completed over its passes, and waits only where the data
// need it: before reading column block x of its input (the ring of the wave
// before it, or for wave 0 of a later round the boundary in HBM) until the
// producer has completed the sub-group that stored it (x + 1 of its pass),
// and before writing ring slot x % 4 until the consumer has read the block
// that slot held (x - 4: the consumer has completed its sub-group x - 4; at
// a pass's first four blocks, the consumer's previous pass up to its last
// ring read: the slots restart at every pass, so the previous occupant is
// not x - 4 across the wrap).  The producer then runs 3 or 4 sub-groups
// ahead of its consumer; nothing waits for the other group of the workgroup
// or for a wave that is not a neighbour.
// Measured (profiles/r05_ab/pair_flags/, same box, two runs each): affine
// gaps C2 +0.3 %, its 1/8 share +0.9 %, 1/4 +0.4 %, wave groups on every
// block +1.6 % against the tick form; the linear cell's cheaper sub-groups
// lost 0.1-0.5 % with the per-sub-group release and count, so linear groups
// keep the tick (the other forms' numbers: profiles/r05_ab/pair_flags/).
template <bool AFFINE>
constexpr bool pair_flags() { return AFFINE; }
struct PairSync {
    int* prog;      // LDS: completed sub-groups of each wave of the workgroup
    int me;         // this wave
    int base;       // this wave's count at the start of this pass (its k-th: k S)
    int pred;       // the wave that produced this pass's input (-1: none)
    int pred_base;  // its count at the start of the pass that produced it
    int succ;       // the wave that reads this pass's ring output (-1: none)
    int S;          // sub-groups per pass
};
__device__ __forceinline__ void pair_wait(const int* prog, int wave, int need) {
    while (__hip_atomic_load(prog + wave, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
        __builtin_amdgcn_s_sleep(1);
}

// One pass (rows [s0, s0 + 2R)) of one 64-subject block.  PAIR: the pass
// is part of a wave pair's pipeline (sw_inter_x2p): the boundary comes from /
// goes to the partner wave through an LDS ring instead of HBM when ring_in /
// ring_out are set, and every sub-group ends with one workgroup barrier (a tick).
//
// CHAIN (single-wave blocks): all passes of the block in ONE sweep over
// npass x ncols virtual columns.  The low strip enters pass k at virtual
// column k ncols while the high strip still finishes pass k-1's last SG
// columns, so the lag sub-group of each pass boundary does useful work in
// both halves (2 % of C2's sub-groups otherwise half idle).  At that
// transition the lo image is restaged and the low halves of H, E and dtop
// restart; SG columns later the same for the hi image and the high halves.
// The low strip's row -1 input of pass k's first columns was stored by pass
// k-1's high strip at least one sub-group earlier (ncols >= 32).
template <int R, int SG, bool AFFINE, bool F16, bool PAIR, int CR = 16, bool CHAIN = false>
__device__ __forceinline__ void x2s_pass(const InterArgs& a, X2Lds<R>& L, uint32_t ncols, uint64_t base, int lane,
                                         int s0, Best<F16>& best, const int4* ring_in, int4* ring_out,
                                         int* tick, const PairSync* ps = nullptr) {
    static_assert(!(CHAIN && PAIR), "chained passes: single-wave blocks only");
    // SG: sub-group width = the lag (columns) between the two strips
    // CR: profile rows per LDS chunk (16: 2 x 4 ds_read_b128 in flight; 8
    // halves the chunk registers)
    constexpr int CQ = CR / 4;
    constexpr int NCH = R / CR;
    constexpr int STEPS = SG * NCH;
    using P = PkCell<F16>;
    using V = typename P::V;
    const int16_t* prof16 = reinterpret_cast<const int16_t*>(a.prof);
    const u2 go2 = {static_cast<unsigned short>(a.gap_open), static_cast<unsigned short>(a.gap_open)};
    const u2 ge2 = {static_cast<unsigned short>(a.gap_extend), static_cast<unsigned short>(a.gap_extend)};
    uint32_t* bnd = reinterpret_cast<uint32_t*>(a.bnd_h);
    // fp16 biased cell constants (exact integers, host-built, SGPRs)
    static_assert(!F16 || (R % kRowGroup == 0 && SG <= 8), "fp16 row groups");
    h2 gog_h = {}, reb_h = {}, grp_h = {};
    if constexpr (F16) {
        gog_h = __builtin_bit_cast(h2, a.f16_gog);
        // unshifted: SG ge (the rebase per sub-group), 16 ge (the row-group reset)
        static_assert(SG == 4 || SG == 8, "rebase constants");
        reb_h = __builtin_bit_cast(h2, a.f16_diff[SG == 4 ? 0 : 1]);
        grp_h = __builtin_bit_cast(h2, a.f16_diff[2]);
    }
    const bool first = (s0 == 0);
    const bool last = (s0 + 2 * R >= a.qpad);
    // CHAIN: passes in this sweep and its virtual width
    const uint32_t npass = CHAIN ? static_cast<uint32_t>((a.qpad + 2 * R - 1) / (2 * R)) : 1u;
    const uint32_t total = npass * ncols;
    const int sbias = F16 ? (AFFINE ? 2 : 1) * a.gap_extend : 0;
    // fp16: the images hold S + 2 ge (the diagonal comes from bias r - 1 + jj - 1;
    // the linear profile already holds S + g); a row group's first row S + 2 ge
    // - 16 ge: its diagonal (the row above, or row -1 from the boundary / delay
    // line) still has the previous row group's bias, and the profile, not an
    // extra subtraction per column, takes it back
    const int gbias0 = F16 ? -kRowGroup * a.gap_extend : 0;
    // packed H of row -1 at the previous step, with the last row group's bias
    const uint32_t dtop0 = F16 ? a.f16_step[SG - 2 + kRowGroup] : 0u;
    stage_x2s<R, F16>(L, prof16, a.prof_stride, s0, lane, sbias, gbias0, -1);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");

    // fp16: cell (r, jj) carries the bias (r % 16 + jj) ge (see the cell
    // below).  Before the first sub-group's rebase the state is that of
    // column SG - 1 of a sub-group: H of column -1 (= 0) is (r % 16 + SG - 1)
    // ge, row -1's H (dtop) (SG - 2) ge; rows come in from the boundary with
    // the last row group's bias, (15 + jj) ge for H and (16 + jj) ge for F.
    V H[R];
    V E[AFFINE ? R : 1];
#pragma unroll
    for (int r = 0; r < R; ++r) H[r] = P::from(F16 ? a.f16_step[r % kRowGroup + SG - 1] : 0u);
#pragma unroll
    for (int r = 0; r < (AFFINE ? R : 1); ++r) E[r] = P::from(F16 ? a.f16_zero : 0u);
    uint32_t dtop = dtop0;             // packed H of row -1 at the previous step
    uint32_t dl_h[SG], dl_f[SG];       // low strip's bottom row, SG steps back
    uint32_t bin[SG], bin_n[SG];       // HBM boundary in (H | F << 16), this / next sub-group
    uint32_t bz[SG];                   // the zero boundary row
    uint32_t rc[SG / 4], rp[SG / 4], rn[SG / 4];  // codes: current (low), previous (high), next
#pragma unroll
    for (int q = 0; q < SG; ++q) {
        // (linear: H of row -1 in both halves, as the 16-bit hand-off loads it)
        bz[q] = !F16 ? 0u
                     : AFFINE ? lo_lo(a.f16_step[kRowGroup - 1 + q], a.f16_step[kRowGroup + q])
                              : lo_lo(a.f16_step[kRowGroup - 1 + q], a.f16_step[kRowGroup - 1 + q]);
        dl_h[q] = F16 ? a.f16_step[kRowGroup - 1 + q] : 0u;
        dl_f[q] = F16 ? a.f16_step[kRowGroup + q] : 0u;
        bin[q] = bz[q];
        bin_n[q] = 0;
    }
#pragma unroll
    for (int q = 0; q < SG / 4; ++q) rp[q] = 0x19191919u;  // virtual columns before the subject
    load_codes<SG>(rc, a.residues + base, true);
    // (flags: column block x of the input is ready once its producer has
    // completed sub-group x + 1 of its pass)
    constexpr bool kPairFlags = pair_flags<AFFINE>();
    auto wait_in = [&](uint32_t x) {
        if constexpr (PAIR && kPairFlags)
            pair_wait(ps->prog, ps->pred, ps->pred_base + min(static_cast<int>(x) + 2, ps->S));
    };
    if (!first) {
        wait_in(0);
        if (PAIR && ring_in) ring_load<SG>(bin, ring_in, 0, lane);
        else load_bnd<SG, AFFINE>(bin, bnd, base);
    }
    int4 PL[2][CQ], PH[2][CQ];
    constexpr uint32_t RB = x2_row_dwords(R) * 4;
    const uint32_t blo = lds_addr(L.lo), bhi = lds_addr(L.hi);
    // LDS addresses of the code rows of the column being prefetched
    uint32_t aa = code_row<RB>(rc, 0, blo), ab = code_row<RB>(rp, 0, bhi);
    read_x2a<CQ>(PL[0], PH[0], aa, ab, 0, 0);

    // sub-groups 0 .. total/SG: the last one runs the high strip only.
    // CHAIN: lo_p / lo_c = the low strip's pass and its first column in that
    // pass (running counters: no divisions in the loop); t2 = the high strip
    // enters a pass (the sub-group after the low strip's entry)
    uint32_t lo_p = 0, lo_c = 0;
    bool t2 = false;
    for (uint32_t col0 = 0; col0 <= total; col0 += SG) {
        const bool has_next = col0 + SG <= total;          // another sub-group follows
        const bool next_lo = col0 + SG < total;            // ... with real low-strip columns
        const uint32_t ncol = col0 + SG;
        const bool wrap = CHAIN && lo_c + SG == ncols;      // the next sub-group starts a pass
        const uint32_t nreal = CHAIN ? (wrap ? 0u : lo_c + SG) : ncol;  // its column in the subject
        const bool next_first = CHAIN ? (lo_p == 0 && !wrap) : first;
        const uint64_t noff = (nreal >> 4) * kGroupBytes + (nreal & 15);
        const bool t1 = CHAIN && lo_c == 0 && lo_p > 0 && lo_p < npass;  // low strip enters pass lo_p
        // the next sub-group starts a pass in the low strip (T1) or the high
        // strip (T2): its first profile words are read after the restaging
        // instead of prefetched here
        const bool next_t1 = CHAIN && wrap && next_lo;
        const bool next_t2 = t1;
        if (t1) {
            stage_x2s<R, F16>(L, prof16, a.prof_stride, static_cast<int>(lo_p) * 2 * R, lane, sbias, gbias0, 0);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                H[r] = P::from(__builtin_amdgcn_perm(P::bits(H[r]), F16 ? a.f16_step[r % kRowGroup + SG - 1] : 0u,
                                                     0x07060100u));
                if constexpr (AFFINE) E[r] = P::from(__builtin_amdgcn_perm(P::bits(E[r]), F16 ? a.f16_zero : 0u, 0x07060100u));
            }
            dtop = __builtin_amdgcn_perm(dtop, dtop0, 0x07060100u);
        }
        if (t2) {
            // the high strip enters pass lo_p (the low strip entered it one sub-group ago)
            stage_x2s<R, F16>(L, prof16, a.prof_stride, static_cast<int>(lo_p) * 2 * R, lane, sbias, gbias0, 1);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                H[r] = P::from(__builtin_amdgcn_perm(F16 ? a.f16_step[r % kRowGroup + SG - 1] : 0u, P::bits(H[r]),
                                                     0x07060100u));
                if constexpr (AFFINE) E[r] = P::from(__builtin_amdgcn_perm(F16 ? a.f16_zero : 0u, P::bits(E[r]), 0x07060100u));
            }
            dtop = __builtin_amdgcn_perm(dtop0, dtop, 0x07060100u);
        }
        if (t1 || t2) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            aa = code_row<RB>(rc, 0, blo);
            ab = code_row<RB>(rp, 0, bhi);
            read_x2a<CQ>(PL[0], PH[0], aa, ab, 0, 0);
        }
        if (next_t1) {
            // pass k's row -1 input: pass k-1's stores of columns 0..SG-1
            // (this wave's own, one or more sub-groups ago) complete first
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
        if (has_next) {
            load_codes<SG>(rn, a.residues + base + noff, next_lo);
            if (!next_first && next_lo) {
                wait_in(ncol / SG);
                if (PAIR && ring_in) ring_load<SG>(bin_n, ring_in, (ncol / SG) % kRingSlots, lane);
                else load_bnd<SG, AFFINE>(bin_n, bnd, base + noff);
            }
        }
        if constexpr (F16) {
            // rebase: column SG-1's bias (SG-1) ge -> column 0's 0, applied to
            // what crosses the sub-group boundary (H as the next diagonal, E)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                H[r] = H[r] - reb_h;
                if constexpr (AFFINE) E[r] = E[r] - reb_h;
            }
            dtop = P::bits(P::from(dtop) - reb_h);
        }
        // One cell pair: row r of column jj.  `up`, `diag` and `f` roll down
        // the column; slo = (S_low strip, 1), shi = (1, S_high strip), so
        // slo * shi + diag is the pair's H_diag + S in one packed op.
        auto cell = [&](const int r, const int jj, V& up, V& diag, V& f, const V slo, const V shi) {
            if constexpr (F16 && !AFFINE) {
                // Biased linear cell: H~ = H + (r % 16 + jj) g, so the left and
                // up terms H - g are the stored neighbours themselves and
                // H~ = max(max3(left, up, H_diag + S + 2 g), floor): 3 packed
                // ops per cell pair + the anti-diagonal maxima.
                const int rg = r % kRowGroup;
                if (rg == 0 && r > 0) up = up - grp_h;  // next row group: its bias restarts at 0
                const h2 t = max3h(H[r], up, __builtin_elementwise_fma(slo, shi, diag));
                const h2 h = __builtin_elementwise_maximum(t, __builtin_bit_cast(h2, a.f16_step[rg + jj]));
                h2& acc = best.acc[rg + jj];
                if (jj & 1) {
                    if (rg + 1 < kRowGroup) acc = max3h(acc, h, H[r + 1]);
                    else acc = __builtin_elementwise_maximum(acc, h);
                } else if (rg == 0) {
                    acc = __builtin_elementwise_maximum(acc, h);
                }
                diag = H[r];
                H[r] = h;
                up = h;
            } else if constexpr (!AFFINE) {
                const s2 h = usub2(max2(max2(H[r], up), slo * shi + diag), go2);
                diag = H[r];
                H[r] = h;
                up = h;
                best.v = max2(best.v, h);
            } else if constexpr (!F16) {  // (fp16 affine: cell_d below)
                const s2 h = max2(max2(E[r], f), slo * shi + diag);
                const s2 n = usub2(h, go2);
                E[r] = max2(usub2(E[r], ge2), n);
                f = max2(usub2(f, ge2), n);
                diag = H[r];
                H[r] = h;
                up = h;
                best.v = max2(best.v, h);
            }
        };
        // The biased Farrar cell (fp16, affine), its diagonal sum d given.
        // Cell (r, jj) holds H~ = H + b, E' = E + b, F~ = F + b with b = (r %
        // 16 + jj) ge, so both gap extensions are the drift of the bias: E' =
        // max(E', m) along the row and F~ = max3(F~, m, floor) down the column
        // with m = H~ - go + ge, no subtraction.  F carries the 0 floor (H >=
        // 0), b of the next row.  5 packed ops per cell pair (+ about half a
        // max3 for the maximum, 2 per row per sub-group for the column rebase,
        // 4 per column for the row-group resets).
        auto cell_d = [&](const int r, const int jj, V& up, V& diag, V& f, const V d) {
          if constexpr (F16 && AFFINE) {
            const int rg = r % kRowGroup;
            if (rg == 0 && r > 0) f = f - grp_h;  // next row group: its bias restarts at 0
            const h2 h = max3h(E[r], f, d);
            const h2 m = h - gog_h;
            E[r] = __builtin_elementwise_maximum(E[r], m);
            f = max3h(f, m, __builtin_bit_cast(h2, a.f16_step[rg + jj + 1]));
            h2& acc = best.acc[rg + jj];
            if (jj & 1) {
                if (rg + 1 < kRowGroup) acc = max3h(acc, h, H[r + 1]);  // H[r + 1]: cell (r + 1, jj - 1)
                else acc = __builtin_elementwise_maximum(acc, h);
            } else if (rg == 0) {  // the even columns' other rows are partners above
                acc = __builtin_elementwise_maximum(acc, h);
            }
            diag = H[r];
            H[r] = h;
            up = h;
          }
        };
        // end of column jj: its bottom row feeds the high strip SG steps later
        auto col_done = [&](const V up, const V f, const int jj) {
            dl_h[jj] = P::bits(up);
            if constexpr (AFFINE) dl_f[jj] = P::bits(f);
        };
        // row -1 inputs of column jj: low strip from HBM (previous pass),
        // high strip from the low strip's bottom row SG steps back (fp16:
        // both from the last row group's bias to row -1's / row 0's)
        auto col_start = [&](V& up, V& diag, V& f, const int jj) {
            // (linear, odd columns: the 16-bit hand-off holds their H in the high half)
            const uint32_t u = (AFFINE || jj % 2 == 0) ? lo_lo(bin[jj], dl_h[jj]) : hi_lo(bin[jj], dl_h[jj]);
            // fp16: row 0's diagonal keeps the last row group's bias (the
            // profile's row 0 takes it back); the linear cell's up term drops it
            up = P::from(u);
            if constexpr (F16 && !AFFINE) up = up - grp_h;
            diag = P::from(dtop);
            dtop = u;
            if constexpr (AFFINE) f = P::from(hi_lo(bin[jj], dl_f[jj]));
            if constexpr (F16) f = f - grp_h;
        };
        V up = P::from(0u), diag = P::from(0u), f = P::from(0u);
#pragma unroll
        for (int t = 0; t < STEPS; ++t) {
            const int jj = t / NCH;
            const int k = t % NCH;
            const uint32_t dep = P::bits(k == 0 ? H[R - 1] : H[CR * k - 1]);
            if (t + 1 < STEPS) {
                const int jn = (t + 1) / NCH, kn = (t + 1) % NCH;
                if (kn == 0) {
                    aa = code_row<RB>(rc, jn, blo);
                    ab = code_row<RB>(rp, jn, bhi);
                }
                read_x2a<CQ>(PL[(t + 1) & 1], PH[(t + 1) & 1], aa, ab, kn, dep);
            } else if (has_next && !next_t1 && !next_t2) {
                aa = code_row<RB>(rn, 0, blo);
                ab = code_row<RB>(rc, 0, bhi);
                read_x2a<CQ>(PL[(t + 1) & 1], PH[(t + 1) & 1], aa, ab, 0, dep);
            }
            if (k == 0) col_start(up, diag, f, jj);
            const int4(&pl)[CQ] = PL[t & 1];
            const int4(&ph)[CQ] = PH[t & 1];
            if constexpr (F16 && AFFINE) {
                // the step's CR diagonal sums first (they read only the old H
                // values), so the dependent chain h -> m -> F of each row has
                // independent work beside it
                V dd[CR];
#pragma unroll
                for (int i = 0; i < CR; ++i)
                    dd[i] = __builtin_elementwise_fma(P::from(word(pl, i)), P::from(word(ph, i)),
                                                      i == 0 ? diag : H[CR * k + i - 1]);
#pragma unroll
                for (int i = 0; i < CR; ++i) asm volatile("" : "+v"(dd[i]));
#pragma unroll
                for (int i = 0; i < CR; ++i) cell_d(CR * k + i, jj, up, diag, f, dd[i]);
            } else {
#pragma unroll
                for (int i = 0; i < CR; ++i)
                    cell(CR * k + i, jj, up, diag, f, P::from(word(pl, i)), P::from(word(ph, i)));
            }
            if (k == NCH - 1) col_done(up, f, jj);
            // pin the running maxima at every step: left free, the compiler
            // defers the max reductions and keeps every h alive (spills)
            if constexpr (!F16) asm volatile("" : "+v"(best.v));
            else best.pin();
            __builtin_amdgcn_sched_barrier(0);
        }
        // the high strip just finished columns [col0 - SG, col0)
        // the high strip's pass: the low strip's, or the one before while
        // the low strip is in its first sub-group
        const bool high_last = CHAIN ? (lo_c == 0 ? lo_p : lo_p + 1) >= npass : last;
        if (!high_last && col0 >= SG) {
            // boundary out = the high halves of the delay line just written
            uint32_t hb[SG];
#pragma unroll
            for (int q = 0; q < SG; ++q) hb[q] = AFFINE ? hi_hi(dl_h[q], dl_f[q]) : hi_hi(dl_h[q], dl_h[q]);
            const uint32_t pc = CHAIN ? (lo_c == 0 ? ncols - SG : lo_c - SG) : col0 - SG;
            if (PAIR && ring_out) {
                // (flags: the slot's previous block has been read: x - 4 of
                // this pass, read before the consumer's sub-group x - 4 ends
                // (block 0 before its pass starts, the others one sub-group
                // ahead), or for x < 4 one of the consumer's previous pass,
                // whose last ring read is in its sub-group S - 3)
                if constexpr (kPairFlags) {
                    const int x = static_cast<int>(pc / SG);
                    pair_wait(ps->prog, ps->succ, x >= kRingSlots ? ps->base + x - kRingSlots + 1 : ps->base - 2);
                }
                ring_store<SG>(ring_out, (pc / SG) % kRingSlots, lane, hb);
            } else {
                const uint64_t poff = (pc >> 4) * kGroupBytes + (pc & 15);
                store_bnd<SG, AFFINE>(bnd, base + poff, hb);
            }
        }
        if (has_next) {
#pragma unroll
            for (int q = 0; q < SG / 4; ++q) {
                rp[q] = rc[q];
                rc[q] = rn[q];
            }
#pragma unroll
            for (int q = 0; q < SG; ++q) bin[q] = (next_first || !next_lo) ? bz[q] : bin_n[q];
        }
        if constexpr (PAIR && kPairFlags) {
            // this sub-group's ring and HBM stores (and its ring reads) are
            // complete before its count
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __hip_atomic_store(ps->prog + ps->me, ps->base + static_cast<int>(col0 / SG) + 1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if constexpr (PAIR) {
            __syncthreads();  // one tick of the pair's clock
            ++*tick;
        }
        if constexpr (CHAIN) {
            t2 = t1;
            lo_c = nreal;
            lo_p += wrap ? 1u : 0u;
        }
    }
}

// A block's width for the fp16 / int16 kernels: the longest subject rounded
// up to 8 columns when the host provides it (the last 16-column group may be
// half used: 8 pad columns fewer per pass for half the blocks, C2 2.1 -> 1.0 %
// of the cells; C2 +1.2 %, C3 +1.0 %, profiles/r03_ab/cols8/).
__device__ __forceinline__ uint32_t block_cols(const InterArgs& a, int blk) {
    return a.blk_cols ? a.blk_cols[blk] : a.blk_groups[blk] * kGroupCols;
}

template <int R, int SG, bool AFFINE, bool F16, int CR>
__device__ __forceinline__ bool x2s_block(const InterArgs& a, int blk, X2Lds<R>& L, int lane) {
    const uint32_t ncols = block_cols(a, blk);
    const uint64_t base = a.blk_off[blk] + static_cast<uint64_t>(lane) * kGroupCols;
    Best<F16> best;
    best.init(a);
    const uint64_t t0 = trace_now();
    if (ncols >= 32 && a.qpad > 2 * R) {
        x2s_pass<R, SG, AFFINE, F16, false, CR, true>(a, L, ncols, base, lane, 0, best, nullptr, nullptr, nullptr);
    } else {
        for (int s0 = 0; s0 < a.qpad && ncols > 0; s0 += 2 * R)
            x2s_pass<R, SG, AFFINE, F16, false, CR>(a, L, ncols, base, lane, s0, best, nullptr, nullptr, nullptr);
    }
    const bool flagged = x2s_finish<F16>(a, blk, lane, best.value(a));
    trace_block(a, blk, t0, lane, 0);
    return flagged;
}

// ---------------------------------------------------------------------------
// sw_inter_x2p: a wave PAIR (or QUAD) per wide block
// ---------------------------------------------------------------------------
// The single-wave kernel runs a block's passes one after another, so a wide
// block's latency is passes x width and the widest blocks (and the last,
// ragged round of short ones) bound the scan (profiles/r01_tail/).  Here the
// G waves of a group (G = 2: a pair, two groups per workgroup; G = 4: a quad,
// the whole workgroup) split the passes: wave w runs passes w, w + G,
// w + 2G, ..., kPairLag sub-groups behind wave w - 1.  Within a round the
// boundary (H | F << 16) goes from wave w to wave w + 1 through an LDS ring;
// from one round to the next (wave G-1 -> wave 0) through HBM as in the
// single-wave kernel.  Linear gaps: all four waves of the workgroup share one
// clock, one __syncthreads per sub-group (below); affine gaps: each wave
// waits only for its neighbours' progress counts (PairSync, above), with the
// same data dependencies.  Schedule of a block whose pass takes
// S = width / SG + 1 ticks: round r of wave w starts at tick
// r * max(S, G kPairLag) + kPairLag w, so
//   * wave w + 1 reads sub-group g of a ring 2 ticks after wave w wrote it and
//     wave w overwrites that slot only 3 ticks after the read (4 slots); a
//     new round's first write comes after the old round's last read;
//   * wave 0 of round r+1 prefetches from HBM what wave G-1 of round r stored
//     at least one tick earlier (period >= G kPairLag).
// Block latency drops from P x S to ceil(P / G) x S + kPairLag (G - 1)
// ticks for P passes; the extra cost is one barrier per sub-group and the
// idle lag.  Pairs take the widest blocks of large databases; quads those of
// small ones (a rank's share of a strong-scaled database), where too few
// blocks exist to fill the GPU and the widest block's latency bounds the
// scan (sw_capi.cpp pair_blocks / pair_group).
constexpr int kPairLag = 3;
// Profile rows per LDS chunk in the group launches (the wave groups' passes
// and the merged launch's single-wave blocks): 8, not the per-wave kernel's
// 16.  These kernels hold 2 waves per SIMD (LDS and the ring buffers) and
// the 16-row double buffer left them 148 B of register spills in the pass
// loop; at 8 rows they spill nothing (C2 10,219 -> 10,320 GCUPS, C3
// 10,323 -> 10,510, the 1/8 share 1.302 -> 1.309 ms per step).  3 waves
// per SIMD does not fit: 168 registers spill 400-800 B.
constexpr int kPairCR = 8;
constexpr int kSingleCR = 8;
constexpr int kGroupWavesPerEU = 2;

__device__ __forceinline__ int group_ticks(uint32_t ncols, int passes, int SG, int G) {
    if (ncols == 0 || passes <= 0) return 0;
    const int S = static_cast<int>(ncols) / SG + 1;
    const int per = max(S, G * kPairLag);
    int t = 0;
    for (int p = max(0, passes - G); p < passes; ++p) t = max(t, (p / G) * per + kPairLag * (p % G) + S);
    return t;
}

// The LDS of one workgroup of the group form: the waves' profile images, the
// rings between consecutive waves of a group (3 for a quad, 2 for two
// pairs), the partial maxima.  53 KB for pairs, 61 KB for quads: both still
// leave 2 workgroups per CU, the register-bound occupancy.
template <int R, int SG, int GMAX>
struct X2pSmem {
    X2Lds<R> lds[kWavesPerWG];
    int4 ring[kWavesPerWG - kWavesPerWG / GMAX][kRingSlots * (SG / 4) * kLanes];
    uint32_t part[kWavesPerWG][kLanes];
    int prog[kWavesPerWG];  // affine groups: completed sub-groups per wave
};

// One workgroup's work (wgi = its index in the launch's numbering):
// workgroups [0, Q) run the Q blocks [blk_base, quad_end) by quads (GMAX = 4
// only), the next ones blocks [quad_end, npair) by pairs (two per
// workgroup), and with MERGED the rest blocks [npair, blk_tail) one per wave
// and the narrowest, [blk_tail, nblocks), by pairs again
// (x2s_block): the dispatcher hands out work widest-first across the forms.
// Returns (per wave) whether this wave appended a block to the rescue list.
template <int R, int SG, bool AFFINE, bool F16, bool MERGED, int GMAX>
__device__ __forceinline__ bool x2p_wg(const InterArgs& a, int wgi, int quad_end, X2pSmem<R, SG, GMAX>& sm) {
    static_assert(R % 16 == 0 && SG % 4 == 0, "shape");
    static_assert(GMAX == 2 || GMAX == 4, "groups of 2 or 4 waves");
    X2Lds<R>* lds = sm.lds;
    auto& ring = sm.ring;
    auto& part = sm.part;
    using P = PkCell<F16>;
    using V = typename P::V;
    const int tid = tid_x();
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int npair = MERGED ? a.blk_first : a.nblocks;  // blocks [blk_base, npair) by groups
    const int qend = GMAX == 4 ? quad_end : a.blk_base;   // blocks [blk_base, qend) by quads
    const int qwg = qend - a.blk_base;                     // quad workgroups
    const int pwg = qwg + (npair - qend + 1) / 2;          // ... and pair workgroups
    // MERGED: blocks [npair, tail) one per wave, then the narrowest blocks
    // [tail, nblocks) by pairs again (the launch's last-dispatched work)
    const int tail = MERGED && a.blk_tail > npair && a.blk_tail < a.nblocks ? a.blk_tail : a.nblocks;
    // 3-wave groups (MERGED, affine gaps, a.blk_tri) instead of quads over
    // [blk_base, qend): a 6-pass block takes two rounds of three passes, no
    // wave idle in the second, and the workgroup's fourth wave (the spare)
    // runs single-wave block npair + wgi — the widest singles beside the
    // widest groups; the single-wave range then starts after them (s0)
    const bool tri_on = MERGED && GMAX == 4 && AFFINE && a.blk_tri != 0;
    const int nspare = tri_on ? max(0, min(qwg, tail - npair)) : 0;
    const int s0 = npair + nspare;
    const int twg = pwg + (tail - s0 + kWavesPerWG - 1) / kWavesPerWG;  // first tail-pair workgroup
    const bool tailp = MERGED && wgi >= twg;               // workgroup-uniform
    if (MERGED && wgi >= pwg && !tailp) {
        const int blk = s0 + (wgi - pwg) * kWavesPerWG + wave;
        // workgroup-uniform branch: no barrier below is skipped by part of it
        return blk < tail && x2s_block<R, SG, AFFINE, F16, kSingleCR>(a, blk, lds[wave], lane);
    }
    const bool quad = !tailp && wgi < qwg;                 // workgroup-uniform
    const bool tri = tri_on && quad;                       // workgroup-uniform
    const bool spare = tri && wave == kWavesPerWG - 1;     // wave-uniform
    const int G = tri ? 3 : quad ? 4 : 2, NG = tri ? 1 : kWavesPerWG / G;
    const int first = quad ? a.blk_base + wgi : tailp ? tail + (wgi - twg) * 2 : qend + (wgi - qwg) * 2;
    const int gend = tailp ? a.nblocks : npair;            // this workgroup's range end
    const int gi = spare ? 0 : wave / G, w = spare ? 0 : wave % G;
    const int passes = (a.qpad + 2 * R - 1) / (2 * R);
    // the workgroup's clock runs to the longest of its blocks
    int tmax = 0;  // (the tick form only)
    for (int q = 0; q < NG; ++q) {
        const int b = first + q;
        if (b < gend) tmax = max(tmax, group_ticks(block_cols(a, b), passes, SG, G));
    }
    const int blk = first + gi;
    Best<F16> best;
    best.init(a);
    int tick = 0;
    const uint64_t t0 = trace_now();
    constexpr bool kPairFlags = pair_flags<AFFINE>();
    if constexpr (kPairFlags) {
        if (tid < kWavesPerWG) sm.prog[tid] = 0;
        __syncthreads();
    }
    bool flagged = false;
    if (spare) {
        const int sb = npair + wgi;  // (x2s_block synchronises with no other wave)
        if (sb < s0) flagged = x2s_block<R, SG, AFFINE, F16, kSingleCR>(a, sb, lds[wave], lane);
    } else if (blk < gend) {
        const uint32_t ncols = block_cols(a, blk);
        const uint64_t base = a.blk_off[blk] + static_cast<uint64_t>(lane) * kGroupCols;
        const int per = max(static_cast<int>(ncols) / SG + 1, G * kPairLag);
        const int4* rin = w > 0 ? ring[gi * (G - 1) + w - 1] : nullptr;
        int4* rout = w < G - 1 ? ring[gi * (G - 1) + w] : nullptr;
        PairSync ps{sm.prog, wave, 0, -1, 0, w < G - 1 ? wave + 1 : -1, static_cast<int>(ncols) / SG + 1};
        for (int p = w; p < passes && ncols > 0; p += G) {
            if constexpr (kPairFlags) {
                // pass p's input: pass p - 1, by the wave before (this round)
                // or by the group's last wave (the round before, in HBM)
                const int k = p / G;
                ps.base = k * ps.S;
                ps.pred = p == 0 ? -1 : w > 0 ? wave - 1 : wave + G - 1;
                ps.pred_base = (w > 0 ? k : k - 1) * ps.S;
            } else {
                const int start = (p / G) * per + kPairLag * w;
                while (tick < start) {
                    __syncthreads();
                    ++tick;
                }
            }
            x2s_pass<R, SG, AFFINE, F16, true, kPairCR>(a, lds[wave], ncols, base, lane, p * 2 * R, best, rin, rout,
                                                        &tick, &ps);
        }
    }
    (void)tmax;
    if constexpr (!kPairFlags) {
        while (tick < tmax) {
            __syncthreads();
            ++tick;
        }
    }
    if (!spare && blk < gend && w > 0) part[wave][lane] = P::bits(best.value(a));
    __syncthreads();
    if (!spare && blk < gend && w == 0) {
        V b = best.value(a);
        for (int u = 1; u < G; ++u) {
            const V o = P::from(part[wave + u][lane]);
            if constexpr (F16) b = __builtin_elementwise_maximum(b, o);
            else b = max2(b, o);
        }
        flagged = x2s_finish<F16>(a, blk, lane, b);
        trace_block(a, blk, t0, lane, tri ? 3 : quad ? 4 : 1);
    }
    return flagged;
}

// G = 2: every group block by pairs; G = 4: every group block by quads.
template <int R, int SG, bool AFFINE, bool F16, bool MERGED, int G>
__global__ __launch_bounds__(256, kGroupWavesPerEU) void sw_inter_x2p(InterArgs a) {
    __shared__ __attribute__((aligned(16))) X2pSmem<R, SG, G> sm;
    x2p_wg<R, SG, AFFINE, F16, MERGED, G>(a, blockIdx.x, MERGED ? a.blk_first : a.nblocks, sm);
}

// ---------------------------------------------------------------------------
// sw_scan_lpt: the inter scan (groups + single waves) and the long subjects'
// fp16 wavefront kernel in ONE launch, longest work first
// ---------------------------------------------------------------------------
// Launched side by side on two streams, the long-subject kernel's workgroups
// are dispatched first and hold slots the inter blocks wait for; on C2 the
// inter launch takes 7.37 ms alone and 7.70 beside it, and on a rank's share
// of a strong-scaled database single-wave blocks start hundreds of us late
// (profiles/r02_strong/traces/).  Here one grid holds both kinds of
// workgroup and order[blockIdx.x] names the work of each: >= 0 an inter
// workgroup of the merged group launch (x2p_wg numbering), < 0 intra
// workgroup -1 - order[..].  The host sorts the table by estimated duration
// (block widths x passes x the tick cost, subject lengths x the step cost),
// so the dispatcher starts the longest work first and fills the end with
// the shortest (LPT).  LDS: the two kinds' buffers overlap (a workgroup is
// one kind), so the occupancy stays the inter kernel's 2 workgroups per CU.
// The drain's shapes: the int16 list form of the two-strips kernel (affine
// 32x8 with 64-row passes, linear 48x4 with 96-row passes) and the int32
// inter kernel (affine 32x8, linear 64x8), as the separate rescue launches.
// The intra forms of the merged launch read lane 0's conveyor inputs from
// LDS under affine gaps (ix2 CONV, 4 KB beside the launch's 57 KB; C2's 1/8
// share +0.6 %; the linear steps, shorter, lost 0.4 % with it and keep the
// readlane form: profiles/r04_ab_lptconv/)

template <bool AFFINE>
struct DrainShape {
    static constexpr int R16 = AFFINE ? 32 : 48, SG16 = AFFINE ? 8 : 4;
    static constexpr int R32 = AFFINE ? 32 : 64;
};
template <bool AFFINE, int RI>
constexpr size_t drain_smem() {
    using D = DrainShape<AFFINE>;
    const size_t x16 = kWavesPerWG * sizeof(X2Lds<D::R16>);
    const size_t i32 = static_cast<size_t>(kProfileRows) * intra_stride(RI);
    const size_t a32 = static_cast<size_t>(kWavesPerWG) * kProfileRows * inter_stride(D::R32);
    const size_t i16 = sizeof(typename ix2::IntraImg<RI, false>::Elem) * ix2::img_elems<RI, false>();
    return std::max(std::max(x16, i32), std::max(a32, i16));
}

// The merged launch's own rescue stages (DrainArgs, sw_kernels.h): after its
// scan work, a workgroup takes entries of the rescue lists until none are
// left — the int16 pairs of list 1 (a whole workgroup: four waves, one LDS
// image), up to four blocks of list A (one int16 block per wave), one subject
// of list 2 (wave 0, int32) or up to four blocks of list B (int32).  A
// workgroup that finds nothing exits; an entry appended later is taken by the
// workgroup that appended it (it drains after appending), so nothing waits
// for other workgroups.  task: 2 + 8 ints of LDS (kind, count, entries).
template <bool AFFINE, int RI>
__device__ __forceinline__ void lpt_drain(const DrainArgs* __restrict__ d, char* smem, int* task) {
    using D = DrainShape<AFFINE>;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    for (;;) {
        __syncthreads();  // the LDS of the previous work is free, task may be rewritten
        if (threadIdx.x == 0) {
            // list 1 first (whole-workgroup work, the longest), then A, 2, B
            constexpr int kOrder[4] = {2, 0, 3, 1};
            constexpr int kWant[4] = {2 * kWavesPerWG, kWavesPerWG, 1, kWavesPerWG};
            int kind = 0, n = 0, start = 0;
            for (int k = 0; k < 4 && !n; ++k) {
                const int l = kOrder[k];
                if ((n = list_claim(d->lists[l], d->heads[l], kWant[k], &start))) kind = l + 1;
            }
            int m = 0;
            for (int i = 0; i < n; ++i) {
                const int v = list_wait_take(d->lists[kind - 1] + 1, start + i, d->fault, d->spin);
                if (v >= 0) task[2 + m++] = v;
            }
            task[0] = m ? kind : (n ? -1 : 0);  // -1: claimed entries never appeared; look again
            task[1] = m;
        }
        __syncthreads();
        const int kind = task[0], n = task[1];
        if (kind == 0) return;  // workgroup-uniform
        if (kind < 0) continue;
        // the producers' results happen-before the re-scoring's stores
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (kind == 3) {  // list 1: int16 pairs, flagging into list 2
            IntraArgs y = d->i16;
            y.subj_list = task + 2;
            y.list_count = task + 1;
            ix2::intra_x2_wg<RI, false, true, !AFFINE, false, false, false, true>(y, 0,
                                                               reinterpret_cast<typename ix2::IntraImg<RI, false>::Elem*>(smem));
        } else if (kind == 1) {  // list A: int16 blocks, flagging into list B
            if (wave < n)
                x2s_block<D::R16, D::SG16, AFFINE, false, 16>(d->a16, task[2 + wave],
                                                              reinterpret_cast<X2Lds<D::R16>*>(smem)[wave], lane);
        } else if (kind == 4) {  // list 2: int32 subject (wave 0)
            if (wave == 0) intra_subject<RI, AFFINE, false>(d->i32, task[2], reinterpret_cast<uint8_t*>(smem));
        } else {  // list B: int32 blocks
            if (wave < n)
                inter_block<D::R32, 8, AFFINE, false>(
                    d->a32, task[2 + wave],
                    reinterpret_cast<uint8_t*>(smem) + wave * (kProfileRows * inter_stride(D::R32)), lane);
        }
    }
}

// The launch's arguments as ONE kernel argument, so that the entry loop
// below can re-read them through an opaque kernarg pointer per entry: read
// as plain kernel arguments, the compiler hoists their loads out of the
// loop and keeps them live across every scan form (169-202 SGPRs of spills).
struct LptParams {
    InterArgs a;
    IntraArgs ia;
    const int32_t* order;
    const DrainArgs* drain;
    int32_t* next;
    int32_t n;
    int32_t grid;  // the launch's workgroups
};

// LOOP = false: one entry per workgroup (entry blockIdx.x), as many
// workgroups as entries.  LOOP = true (a table of many rounds of workgroups):
// one workgroup per resident slot, each taking its next entry from the
// counter `next` once it has finished one — the dispatcher's gaps between
// a workgroup's end and the next one's start on a CU (median 27 us in
// C2's launch, 2 % of its slots idle, profiles/r05_trace/) go away.  The
// loop costs registers: the loop-invariant parts of every scan form (lane
// and LDS addresses) are hoisted out of it and live across all forms
// (+20 VGPRs; under affine gaps 124-156 bytes per lane of spills, outside
// the inner loops), which a launch of few rounds does not win back: C2
// +1.7 % looping against -1.2 % for the looped code run one entry per
// workgroup; the 1/8 share (1.7 rounds) -0.6 % (profiles/r05_ab/lpt_loop/).
// (A noinline entry function instead of the inlined forms faulted on the
// GPU; not pursued.)
template <int R, int SG, bool AFFINE, int RI, bool LOOP>
__global__ __launch_bounds__(256, kGroupWavesPerEU) void sw_scan_lpt(LptParams prm) {
    using Elem = typename ix2::IntraImg<RI, true>::Elem;
    using PElem = typename ix2::IntraImg<2, true>::Elem;
    constexpr size_t kInter = sizeof(X2pSmem<R, SG, 4>);
    constexpr size_t kIntra = sizeof(Elem) * ix2::img_elems<RI, true>();
    constexpr size_t kPipe = kWavesPerWG * sizeof(PElem) * ix2::img_elems<2, true>() + kWavesPerWG * sizeof(int);
    constexpr size_t kDrain = drain_smem<AFFINE, RI>();
    constexpr size_t kSmem = std::max(std::max(std::max(kInter, kIntra), kDrain), kPipe);
    __shared__ __attribute__((aligned(16))) char smem[kSmem];
    __shared__ int task[2 + 2 * kWavesPerWG];
    __shared__ int claimed;
    // Entry k of the table: this workgroup's own index first; then (LOOP)
    // the entry after the grid's that the counter hands out, until the
    // table is exhausted.  Every wave leaves the loop on the same k (LDS).
    if (static_cast<int>(blockIdx.x) >= prm.n) return;
    for (int k = blockIdx.x;;) {
        auto kp = __builtin_amdgcn_kernarg_segment_ptr();
        if constexpr (LOOP) asm volatile("" : "+s"(kp));  // opaque: the arguments are loaded per entry
        const LptParams& p = *(const LptParams*)(kp);     // (C cast: the address-space cast)
        const InterArgs& a = p.a;
        const IntraArgs& ia = p.ia;
        // intra items: -1 - g; g < the launch's intra workgroups (RI rows per
        // lane, 4 pairs) or, past them, one of the longest pairs in the
        // pipelined form (2 rows per lane, a chunk per wave)
        const int niwg = ((ia.nsubj + 1) / 2 + kWavesPerWG - 1) / kWavesPerWG;
        const int item = p.order[k];
        const uint64_t t0 = trace_now();
        bool flagged;
        if (item >= 0)
            flagged = x2p_wg<R, SG, AFFINE, true, true, 4>(a, item, a.blk_quad,
                                                           *reinterpret_cast<X2pSmem<R, SG, 4>*>(smem));
        else if (-1 - item < niwg)
            flagged = ix2::intra_x2_wg<RI, true, false, !AFFINE, true, false, AFFINE, true>(
                ia, -1 - item, reinterpret_cast<Elem*>(smem));
        else
            flagged = ix2::intra_x2_wg<2, true, false, !AFFINE, true, true, AFFINE, true>(
                ia, -1 - item - niwg, reinterpret_cast<PElem*>(smem));
        // Only a workgroup that appended an entry drains (and takes whatever is
        // listed, its own entries included): every entry is then taken by its
        // producer at the latest, and the rest of the grid pays one barrier.
        const bool any = __syncthreads_or(flagged);
        // per-entry timeline (trace builds), after the per-block entries:
        // every wave of the workgroup is done here
        if (threadIdx.x == 0) trace_block(a, a.nblocks + k, t0, 0, item >= 0 ? 2 : 3);
        if (p.drain && any) lpt_drain<AFFINE, RI>(p.drain, smem, task);
        if constexpr (!LOOP) break;
        if (threadIdx.x == 0) claimed = p.grid + __hip_atomic_fetch_add(p.next, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();  // (also: every wave is done with the LDS of this entry)
        k = claimed;
        __syncthreads();  // claimed is read before the next entry's thread 0 rewrites it
        if (k >= p.n) break;
    }
}

// Resident workgroups of sw_scan_lpt<...> on the device (the looped grid):
// occupancy (per CU, once per instantiation: the code object's, the same on
// every device of the build's one architecture) x the handle's CUs.
template <int R, int RI, bool AFFINE>
static int lpt_slots(int cus) {
    static const int per = [] {
        int p = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&p, sw_scan_lpt<R, 8, AFFINE, RI, true>,
                                                         kWavesPerWG * kLanes, 0) != hipSuccess)
            return 0;
        return p;
    }();
    return cus * per;
}

// The looped form from this many rounds of resident workgroups on.
constexpr int kLptLoopRounds = 3;

template <int R, int RI, bool AFFINE>
static void launch_lpt_t(const InterArgs& a, const IntraArgs& ia, const int32_t* order, int n, int cus,
                         hipStream_t s, const DrainArgs* drain, int32_t* next, int loop_grid) {
    int slots = next ? lpt_slots<R, RI, AFFINE>(cus) : 0;
    const dim3 block(kWavesPerWG * kLanes);
    if (next && loop_grid > 0) slots = std::min(loop_grid, n);  // forced (tests)
    if (slots > 0 && (n >= kLptLoopRounds * slots || (next && loop_grid > 0))) {
        const LptParams p{a, ia, order, drain, next, n, slots};
        hipLaunchKernelGGL((sw_scan_lpt<R, 8, AFFINE, RI, true>), dim3(slots), block, 0, s, p);
    } else {
        const LptParams p{a, ia, order, drain, nullptr, n, n};
        hipLaunchKernelGGL((sw_scan_lpt<R, 8, AFFINE, RI, false>), dim3(n), block, 0, s, p);
    }
}

bool lpt_supported(int ri) { return ri == 4 || ri == 6 || ri == 8; }

hipError_t launch_scan_lpt(const InterArgs& a, const IntraArgs& ia, const int32_t* order, int n, bool affine, int ri,
                           int cus, hipStream_t s, const DrainArgs* drain, int32_t* next, int loop_grid, int rows) {
    if (n <= 0) return hipSuccess;
    if ((rows != 64 && rows != 96) || (rows == 96 && affine) || a.qpad % rows) return hipErrorInvalidValue;
#define SW_LPT_RI(RI)                                                                          \
    (affine ? launch_lpt_t<32, RI, true>(a, ia, order, n, cus, s, drain, next, loop_grid)           \
     : rows == 96 ? launch_lpt_t<48, RI, false>(a, ia, order, n, cus, s, drain, next, loop_grid)   \
                  : launch_lpt_t<32, RI, false>(a, ia, order, n, cus, s, drain, next, loop_grid))
    if (ri == 4) SW_LPT_RI(4);
    else if (ri == 6) SW_LPT_RI(6);
    else if (ri == 8) SW_LPT_RI(8);
    else return hipErrorInvalidValue;
#undef SW_LPT_RI
    return hipGetLastError();
}

// merged = false: blocks [a.blk_base, a.nblocks) by wave groups (the caller
// passes the group range's end as nblocks).  merged = true: the whole scan in
// one launch, blocks [a.blk_base, a.blk_first) by groups and [a.blk_first,
// a.nblocks) one per wave.  The two-strips 32x8 shapes only.
template <bool M, int G>
static hipError_t launch_x2p(const InterArgs& a, bool affine, bool f16, hipStream_t s) {
    constexpr int NG = kWavesPerWG / G;
    const int np = M ? a.blk_first : a.nblocks;
    const int nwg = (np - a.blk_base + NG - 1) / NG + (M ? (a.nblocks - np + kWavesPerWG - 1) / kWavesPerWG : 0);
    if (nwg <= 0) return hipSuccess;
    const dim3 grid(nwg), block(kWavesPerWG * kLanes);
    if (f16 && affine) hipLaunchKernelGGL((sw_inter_x2p<32, 8, true, true, M, G>), grid, block, 0, s, a);
    else if (f16) hipLaunchKernelGGL((sw_inter_x2p<32, 8, false, true, M, G>), grid, block, 0, s, a);
    else if (affine) hipLaunchKernelGGL((sw_inter_x2p<32, 8, true, false, M, G>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((sw_inter_x2p<32, 8, false, false, M, G>), grid, block, 0, s, a);
    return hipGetLastError();
}

hipError_t launch_inter_x2p(const InterArgs& a, bool affine, bool f16, bool merged, int group, hipStream_t s) {
    if (a.nblocks <= 0 || a.qpad <= 0) return hipSuccess;
    if (group == 4) return merged ? launch_x2p<true, 4>(a, affine, f16, s) : launch_x2p<false, 4>(a, affine, f16, s);
    if (group != 2) return hipErrorInvalidValue;
    return merged ? launch_x2p<true, 2>(a, affine, f16, s) : launch_x2p<false, 2>(a, affine, f16, s);
}

template <int R, int SG>
static hipError_t launch_x2s_shape(const InterArgs& a, bool affine, hipStream_t s) {
    const dim3 grid((a.nblocks - a.blk_first + kWavesPerWG - 1) / kWavesPerWG), block(kWavesPerWG * kLanes);
    if (affine) hipLaunchKernelGGL((sw_inter_x2s<R, SG, true, false, false>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((sw_inter_x2s<R, SG, false, false, false>), grid, block, 0, s, a);
    return hipGetLastError();
}

hipError_t launch_inter_x2s(const InterArgs& a, int R, int SG, bool affine, bool f16, hipStream_t s) {
    if (a.nblocks - a.blk_first <= 0 || a.qpad <= 0) return hipSuccess;
    if (f16) {
        if (!(R == 32 && (SG == 8 || (SG == 4 && affine)))) return hipErrorInvalidValue;
        const dim3 grid((a.nblocks - a.blk_first + kWavesPerWG - 1) / kWavesPerWG), block(kWavesPerWG * kLanes);
        if (!affine) hipLaunchKernelGGL((sw_inter_x2s<32, 8, false, true, false>), grid, block, 0, s, a);
        else if (SG == 8) hipLaunchKernelGGL((sw_inter_x2s<32, 8, true, true, false>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((sw_inter_x2s<32, 4, true, true, false, 8>), grid, block, 0, s, a);
        return hipGetLastError();
    }
    if (R == 32 && SG == 8) return launch_x2s_shape<32, 8>(a, affine, s);
    return hipErrorInvalidValue;
}

// The int16 packed kernel over a device-side block list (fp16 rescue stage 2):
// a fixed grid walks the list; an empty list costs one tiny launch.
hipError_t launch_inter_x2s_list(const InterArgs& a, bool affine, hipStream_t s) {
    if (a.qpad <= 0) return hipSuccess;
    const dim3 grid(64), block(kWavesPerWG * kLanes);
    if (affine) hipLaunchKernelGGL((sw_inter_x2s<32, 8, true, false, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((sw_inter_x2s<48, 4, false, false, true>), grid, block, 0, s, a);
    return hipGetLastError();
}

}  // namespace swk
