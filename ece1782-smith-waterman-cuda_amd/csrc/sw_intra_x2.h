// sw_intra_x2.h — the body of the two-subjects-per-wave intra-sequence
// kernel (sw_intra_x2.hip), shared with the merged scan launch
// (sw_inter_x2.hip, sw_scan_lpt).
//
// The kernel: intra-sequence wavefront, TWO subjects per wave, packed
// fp16 cell (the long-subject path; config C5).
//
// The anti-diagonal wavefront of sw_intra (sw_kernels.hip): lane t owns query
// rows [c0 + t·RI, c0 + (t+1)·RI) of a 64·RI-row chunk and handles column
// k − t at step k; the bottom row (H, F) and the residue codes move one lane
// per step with DPP wave_shr:1, lane 0 is fed from the previous chunk pass's
// boundary row, lane 63's output is collected for the next pass.  Here every
// value is a PAIR: the low fp16 half belongs to subject 2p, the high half to
// subject 2p+1 (adjacent in the length-sorted order, so their lengths are
// close; the shorter one runs pad columns, score 0, to the longer one's end).
// The cell is the two-strips kernel's (sw_inter_x2.hip) Farrar form on
// v_pk_add_f16 / v_pk_maximum3_f16, so linear gaps run it with open = extend:
//   h = max3(E, F, H_diag + S);  n = h − go;
//   E = max3(E − ge, n, 0);      F = max3(F − ge, n, 0)
// and the substitution pair is one v_perm_b32 of the two subjects' profile
// words.  The four waves of a workgroup share one fp16 image of the chunk's
// profile in LDS, [code][4-row quarter][lane][4 halves]: a lane's quarter is
// 8 bytes at lane·8 within a 512-byte row, so a ds_read_b64 is bank-conflict
// free whatever code each lane reads.  The waves stage each chunk together
// and meet at one barrier per chunk (their subjects have near-equal lengths).
//
// Exactness: fp16 holds every integer up to 2048 (the cells are offset by
// -2048 + 2 ge, so stored values span 4096).  H grows by at most max S per
// cell and the biased values sit up to intra_bias_rows(RI) = max(26, RI +
// period + 2) ge above the true ones (the bias period is 8 steps, 16 at the
// widest shape, RI 20: half the rebases), so a subject whose running maximum reaches
// a.sat_limit = 4096 − 2 ge − 2·max S − intra_bias_rows(RI)·ge (computed
// exactly) is appended to a.rescue_list.
// The same kernel in int16 (IntraCell<false>, LIST) re-scores that list and
// appends subjects near 32767 to a second list for the int32 sw_intra; when
// the fp16 pass would flag most subjects (cheap linear gaps on long pairs)
// the host runs the int16 form first over all of them (sw_capi.cpp).
#pragma once

#include <type_traits>

#include "sw_kernels.h"

namespace swk {
namespace ix2 {

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ h2 hmax3(h2 a, h2 b, h2 c) {
    return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}
__device__ __forceinline__ uint32_t f16_bits(int v) {
    return static_cast<uint32_t>(__builtin_bit_cast(uint16_t, static_cast<_Float16>(v)));
}

// DPP wave_shr:1 (lane t gets lane t-1's value; lane 0 keeps `old`)
__device__ __forceinline__ uint32_t shr1u(uint32_t old, uint32_t src) {
    return static_cast<uint32_t>(
        __builtin_amdgcn_update_dpp(static_cast<int>(old), static_cast<int>(src), 0x138, 0xf, 0xf, false));
}

constexpr int kCodes = kPadCode + 1;  // residue codes 0..24 and the pad code

// fp16 pair of two int16 profile entries minus `b`
__device__ __forceinline__ uint32_t f16x2_of(uint32_t w, int b0, int b1) {
    return f16_bits(static_cast<int16_t>(w & 0xffffu) - b0) | (f16_bits(static_cast<int16_t>(w >> 16) - b1) << 16);
}

typedef short s2 __attribute__((ext_vector_type(2)));

// The cell's number format.  F16: exact integers up to 2048 (the default);
// int16: up to 32767 (the rescue stage for subjects whose fp16 maximum nears
// 2048, e.g. linear scoring with cheap gaps), wrapping add, no 3-input max.
template <bool F16>
struct IntraCell {
    using V = h2;
    static __device__ __forceinline__ V from(uint32_t x) { return __builtin_bit_cast(h2, x); }
    static __device__ __forceinline__ uint32_t bits(V x) { return __builtin_bit_cast(uint32_t, x); }
    static __device__ __forceinline__ V max2(V a, V b) { return __builtin_elementwise_maximum(a, b); }
    static __device__ __forceinline__ V max3(V a, V b, V c) { return hmax3(a, b, c); }
    // the cell values carry the offset zero (IntraArgs::f16_zero): step(j) =
    // (j ge + zero); diff(j) = (j ge), for the rebase and the hand-off drops,
    // is step(j) - step(0) (exact: small integers)
    static __device__ __forceinline__ uint32_t step(const IntraArgs& a, int j) { return a.f16_step[j]; }
    static __device__ __forceinline__ uint32_t diff(const IntraArgs& a, int j) {
        return __builtin_bit_cast(uint32_t, __builtin_bit_cast(h2, a.f16_step[j]) - __builtin_bit_cast(h2, a.f16_step[0]));
    }
    static __device__ __forceinline__ uint32_t zero(const IntraArgs& a) { return a.f16_zero; }
    static __device__ __forceinline__ int zero_int(const IntraArgs& a) {
        return static_cast<int>(static_cast<float>(__builtin_bit_cast(h2, a.f16_zero).x));
    }
    static __device__ __forceinline__ uint32_t pair_of(int v) { const uint32_t b = f16_bits(v); return b | (b << 16); }
    static __device__ __forceinline__ uint32_t convert(uint32_t w, int b0, int b1) { return f16x2_of(w, b0, b1); }
    static __device__ __forceinline__ int lo(V x) { return static_cast<int>(static_cast<float>(x.x)); }
    static __device__ __forceinline__ int hi(V x) { return static_cast<int>(static_cast<float>(x.y)); }
    template <int RI>
    static __device__ __forceinline__ bool flag(const IntraArgs& a, int b) { return b >= a.sat_limit; }
};
template <>
struct IntraCell<false> {
    using V = s2;
    static __device__ __forceinline__ V from(uint32_t x) { return __builtin_bit_cast(s2, x); }
    static __device__ __forceinline__ uint32_t bits(V x) { return __builtin_bit_cast(uint32_t, x); }
    static __device__ __forceinline__ V max2(V a, V b) { return __builtin_elementwise_max(a, b); }
    static __device__ __forceinline__ V max3(V a, V b, V c) { return max2(max2(a, b), c); }
    static __device__ __forceinline__ uint32_t step(const IntraArgs& a, int j) { return pair_of(j * a.gap_extend); }
    static __device__ __forceinline__ uint32_t diff(const IntraArgs& a, int j) { return step(a, j); }
    static __device__ __forceinline__ uint32_t zero(const IntraArgs&) { return 0u; }
    static __device__ __forceinline__ int zero_int(const IntraArgs&) { return 0; }
    static __device__ __forceinline__ uint32_t pair_of(int v) {
        const uint32_t b = static_cast<uint16_t>(v);
        return b | (b << 16);
    }
    static __device__ __forceinline__ uint32_t convert(uint32_t w, int b0, int b1) {
        return static_cast<uint16_t>(static_cast<int16_t>(w & 0xffffu) - b0) |
               (static_cast<uint32_t>(static_cast<uint16_t>(static_cast<int16_t>(w >> 16) - b1)) << 16);
    }
    static __device__ __forceinline__ int lo(V x) { return x.x; }
    static __device__ __forceinline__ int hi(V x) { return x.y; }
    // the int16 guard band (the biased values sit up to max(26, RI + 10) ge
    // above the true ones)
    template <int RI>
    static __device__ __forceinline__ bool flag(const IntraArgs& a, int b) {
        return b >= kSat16 - intra_bias_rows(RI) * a.gap_extend || b < 0;
    }
};

// A lane's rows of one code in the LDS image, 4 rows (int2) per element when
// RI is a multiple of 4 (one ds_read_b64), 2 rows (one dword, ds_read_b32)
// otherwise; either way lane l's element sits at l·size in a 64-element row,
// so the reads are conflict-free whatever code each lane reads.
template <int RI, bool F16>
struct IntraImg {
    static constexpr int kRows = RI % 4 == 0 ? 4 : 2;
    using Elem = typename std::conditional<kRows == 4, int2, uint32_t>::type;
    using LElem = __attribute__((address_space(3))) const Elem;
    static constexpr int kPer = RI / kRows;  // elements per lane and code
    static __device__ __forceinline__ uint32_t word(const Elem (&w)[kPer], int r) {
        if constexpr (kRows == 4) return static_cast<uint32_t>((r & 2) ? w[r >> 2].y : w[r >> 2].x);
        else return w[r >> 1];
    }
    // staging: the element of rows [4q, 4q + 4) or [2q, 2q + 2) of a lane
    // (b0: the first row's drop, b the others')
    static __device__ __forceinline__ Elem load(const int16_t* p, int b0, int b) {
        using C = IntraCell<F16>;
        if constexpr (kRows == 4) {
            const int2 v = *reinterpret_cast<const int2*>(p);
            return make_int2(static_cast<int>(C::convert(static_cast<uint32_t>(v.x), b0, b)),
                             static_cast<int>(C::convert(static_cast<uint32_t>(v.y), b, b)));
        } else {
            return C::convert(*reinterpret_cast<const uint32_t*>(p), b0, b);
        }
    }
};

// LIST: the rescue stage — subject pairs come from the device-side list of
// the subjects the fp16 pass flagged (a.subj_list / a.list_count); the grid
// covers the longest possible list and surplus workgroups return at once.
// Every step reads the NEXT step's profile words from LDS (its codes are
// known one step ahead), so the LDS latency is hidden even when the SIMD's
// waves run in lockstep (C5 7,553 -> 7,609 GCUPS, profiles/r01_prefetch/).

// The LDS image of one chunk: [code][element][lane] (img_elems(RI) elements).
template <int RI, bool F16>
__host__ __device__ constexpr int img_elems() { return kCodes * IntraImg<RI, F16>::kPer * kLanes; }

// One workgroup's work (wgi = its index in the launch: subject pairs
// 4 wgi .. 4 wgi + 3, one per wave); img: the workgroup's LDS image.
// LIN (linear gaps, open == extend = g): the biased cell needs no E or F —
// the left and up terms H - g ARE the stored neighbours (the bias grows by g
// per row and per step), so h~ = max(max3(H~_left, H~_up, H~_diag + S + 2g),
// floor): 2 packed ops per cell pair after the diagonal sum instead of the
// Farrar form's 6 (the two-strips kernel's linear cell, sw_inter_x2.hip).
// TAKE (LIST): the entries are read from the device list and reset (list_take);
// otherwise a.subj_list holds plain subject indices (the merged launch's
// drain passes the entries it took, in LDS).
// Returns (per wave) whether the wave appended a subject to a.rescue_list.
// PIPE (fp16 only, not LIST): ONE subject pair per workgroup (pair wgi), its
// query chunks (at most kWavesPerWG) pipelined over the waves, each wave with
// its own image in img (kWavesPerWG images, then kWavesPerWG progress ints):
// the longest subjects' latency form for the merged launch, whose span one
// long pair otherwise sets (chunks x steps on one wave; here ~steps + 128 per
// extra chunk).
// Staging of the chunk's bottom row (intra_x2_wg): kStage slots per wave
// plus NB scratch slots every lane but 63 writes, 8 bytes each (H, F): one
// LDS array per kernel, whichever forms of intra_x2_wg it instantiates.
// (Stored by lane 63 at every step under an exec mask, with the column's
// range test, the stores cost a lone wave ~16 scalar instructions per step:
// the reference scoring's 1/8 share 10,986 -> 11,975 GCUPS, C5 8,045 ->
// 8,177; 1 KB of LDS, so sw_intra_x2<16> still fits 3 workgroups per CU.)
constexpr int kStage = 32;
__device__ __forceinline__ uint2* bottom_stage() {
    __shared__ uint2 slots[kWavesPerWG * kStage + 8];
    return slots;
}

// CONV: lane 0's conveyor inputs of each step (the boundary row's H and F,
// the code row offsets) come from LDS, one broadcast ds_read_b32 each,
// instead of a v_readlane of the block's register and a v_mov of it back to
// a VGPR for the DPP shift (6 VALU per step): per wave 256 words, [H 64][F
// 64][codes of this block 64][of the next 64], written at each 64-step
// block's start.
constexpr int kConvWords = 256;
__device__ __forceinline__ uint32_t* conv_area() {
    __shared__ uint32_t w[kWavesPerWG * kConvWords];
    return w;
}

template <int RI, bool F16, bool LIST, bool LIN = false, bool TAKE = true, bool PIPE = false,
          bool CONV = false, bool OPQ = false>
__device__ __forceinline__ bool intra_x2_wg(const IntraArgs& a, int wgi, typename IntraImg<RI, F16>::Elem* img) {
    static_assert(!(PIPE && LIST), "the pipelined form takes its pair by index");
    static_assert(RI % 2 == 0 && RI <= kIntraX2MaxRI, "rows per lane");
    constexpr int CH = kLanes * RI;  // query rows per chunk
    using C = IntraCell<F16>;
    using V = typename C::V;
    using Img = IntraImg<RI, F16>;
    using Elem = typename Img::Elem;
    constexpr int NQ = Img::kPer;    // image elements per lane and code
    constexpr int NB = intra_period(RI);  // steps per bias period (one rebase each)
    constexpr int NACC = RI + NB - 1;
    static_assert(RI + NB + 1 <= kIntraSteps, "f16_step table");
    // profile prefetch distance in steps: the pipelined form's short affine
    // steps (RI 2) do not cover an LDS read's latency on a busy CU with one
    // (C2's 1/8 share +0.6 %; linear steps lost 3 % with 2, 6 % with 3)
    constexpr int PF = PIPE && !LIN ? 2 : 1;
    constexpr int NBUF = PF == 1 ? 2 : 4;
    static_assert(PF >= 1 && PF <= NBUF - 1, "prefetch distance");
    // OPQ (the merged launch's looped form): the thread index read opaquely
    // (sw_kernels.h tid_x); the stand-alone kernel reads it plainly (C5: the
    // opaque read cost 0.3 VALU per wave-step)
    const int tid = OPQ ? tid_x() : static_cast<int>(threadIdx.x);
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const bool is_last_lane = lane == kLanes - 1;
    const int p = PIPE ? wgi : wgi * kWavesPerWG + wave;  // subject pair
    int sa = 2 * p, sb = 2 * p + 1;
    // (pairs the merged launch runs in the pipelined form are skipped here)
    const bool skip = !PIPE && !LIST && (p < a.pipe_pairs || p >= a.pipe_tail);
    bool hasA = !skip && sa < a.nsubj, hasB = !skip && sb < a.nsubj;
    if constexpr (LIST) {
        const int n = __builtin_amdgcn_readfirstlane(*a.list_count);
        if (wgi * 2 * kWavesPerWG >= n) return false;  // workgroup-uniform
        hasA = sa < n;
        hasB = sb < n;
        if constexpr (TAKE) {
            sa = hasA ? list_take(a.subj_list, sa) : 0;
            sb = hasB ? list_take(a.subj_list, sb) : 0;
        } else {
            sa = hasA ? a.subj_list[sa] : 0;
            sb = hasB ? a.subj_list[sb] : 0;
        }
    }
    const int LA = hasA ? a.subj_len[sa] : 0;
    const int LB = hasB ? a.subj_len[sb] : 0;
    const int L = max(LA, LB);  // = LA (length-sorted), kept general
    const uint64_t offA = hasA ? a.subj_off[sa] : 0;
    const uint8_t* __restrict__ resA = a.residues + offA;
    const uint8_t* __restrict__ resB = a.residues + (hasB ? a.subj_off[sb] : 0);
    // the pair's boundary rows live in the longer subject's slots
    uint32_t* bnd_h = reinterpret_cast<uint32_t*>(a.bnd_h) + (LA >= LB ? offA : (hasB ? a.subj_off[sb] : 0));
    uint32_t* bnd_f = reinterpret_cast<uint32_t*>(a.bnd_f) + (LA >= LB ? offA : (hasB ? a.subj_off[sb] : 0));
    const int16_t* prof16 = reinterpret_cast<const int16_t*>(a.prof);
    auto step = [&](int j) { return C::from(C::step(a, j)); };  // (j ge, j ge) + the offset
    auto diff = [&](int j) { return C::from(C::diff(a, j)); };  // (j ge, j ge)
    const V gog = C::from(C::pair_of(a.gap_open - a.gap_extend));
    // Biased cell (the two-strips kernel's, sw_inter_x2.hip): at step k,
    // row i of a lane holds H~ = H + (i + k % NB) ge, E' and F~ likewise, so
    // both gap extensions are the drift of the bias:
    //   h = max3(E', F~, H_diag + S + 2 ge);  m = h - (go - ge)
    //   E' = max(E', m);  F~ = max3(F~, m, (i + 1 + k % NB) ge)
    // The bias is a function of the step, the same in every lane, so every
    // NB steps all lanes rebase together (H, E' and the row -1 diagonal
    // drop NB ge), and what crosses lanes (the bottom row's H and F, one step
    // old) drops (RI - 1) ge (+ NB ge at a rebase step).  Maxima per
    // anti-diagonal i + k % NB, two cells per v_pk_maximum3_f16.
    V acc[NACC];
#pragma unroll
    for (int q = 0; q < NACC; ++q) acc[q] = C::from(C::zero(a));

    // One chunk pass: rows [c0, c0 + CH) against the pair's columns, its
    // profile image in cimg; for_blocks(nblk, block) runs block(bk) for the
    // blocks of 64 steps (in order: at once, or one per round of a pipeline).
    auto run_chunk = [&](int c0, Elem* cimg, bool first, bool last, auto&& for_blocks) {
        (void)c0;
            // state of step -1 (column -1 - lane: H = 0), before step 0's rebase
            V H[RI], E[LIN ? 1 : RI];
#pragma unroll
            for (int r = 0; r < RI; ++r) {
                H[r] = step(r + NB - 1);
                if constexpr (!LIN) E[r] = C::from(C::zero(a));
            }
            // bottom row (H, F) of this lane one step back, and H of the row above
            // at the previous column (row 0's diagonal): zeros of step -1
            uint32_t hl = C::step(a, RI + NB - 2), fl = C::step(a, RI + NB - 1);
            // (affine: up_prev is held (RI - 1) ge high, the drop the row-0
            // profile words carry instead, see the hand-off below)
            uint32_t up_prev = C::step(a, LIN ? NB - 2 : NB - 2 + RI - 1);
            // The code conveyor carries the LDS byte offsets of the two
            // subjects' profile rows, A | B << 16 (code x the image's bytes per
            // code, < 2^16): a row address is then one add of a 16-bit field
            constexpr uint32_t kCodeBytes = NQ * kLanes * sizeof(Elem);
            static_assert((kCodes - 1) * kCodeBytes < 0x10000u, "16-bit row offsets");
            constexpr uint32_t kPadPair = kPadCode * kCodeBytes | (kPadCode * kCodeBytes) << 16;
            uint32_t rc = kPadPair;        // row offsets (A | B << 16) of this lane's current column
            uint32_t in_res = kPadPair, in_bh = 0, in_bf = 0;
            const int nsteps = L + kLanes - 1;
            // LDS byte address of this lane's element of code 0
            const uint32_t lrow = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(cimg + lane));

            // the profile words of row offsets rcx (A | B << 16) for this lane
            auto read_words = [&](uint32_t rcx, Elem (&wa)[NQ], Elem (&wb)[NQ]) {
                typename Img::LElem* pa = reinterpret_cast<typename Img::LElem*>(
                    static_cast<uintptr_t>(lrow + (rcx & 0xffffu)));
                typename Img::LElem* pb = reinterpret_cast<typename Img::LElem*>(
                    static_cast<uintptr_t>(lrow + (rcx >> 16)));
#pragma unroll
                for (int qq = 0; qq < NQ; ++qq) {
                    wa[qq] = __builtin_bit_cast(Elem, pa[qq * kLanes]);
                    wb[qq] = __builtin_bit_cast(Elem, pb[qq * kLanes]);
                }
            };
            auto codes_at = [&](int col) {
                const uint32_t ca = col < LA ? resA[col] : kPadCode;
                const uint32_t cb = col < LB ? resB[col] : kPadCode;
                return ca * kCodeBytes | (cb * kCodeBytes) << 16;
            };
            uint32_t in_res_nb = codes_at(lane);  // row offsets of the next block of 64 steps
            // profile words, in NBUF buffers by step (NB is a multiple of NBUF,
            // so a bias period starts on buffer 0): step b reads W[b % NBUF]
            // and prefetches step b + PF's into another, no register copies
            Elem W[NBUF][2][NQ];
            uint32_t rcq[PF];  // codes (lane's column) of steps + 1 .. + PF
#pragma unroll
            for (int d = 0; d < PF; ++d) rcq[d] = 0;

            const int nblk = (nsteps + kLanes - 1) / kLanes;
            // lane 63's bottom row (H, F) of each step goes to its wave's
            // staging slots in LDS (step m: slot m % kStage); every other lane
            // writes the scratch slots, so the per-step store needs no exec
            // mask, no range test and no branch; every kStage steps the wave
            // copies the slots to the boundary row with one coalesced store
            using Slot = typename std::conditional<LIN, uint32_t, uint2>::type;
            Slot* const stg = reinterpret_cast<Slot*>(bottom_stage()) + wave * kStage;
            Slot* const scratch = reinterpret_cast<Slot*>(bottom_stage()) + kWavesPerWG * kStage;
            uint32_t* const cv = CONV ? conv_area() + wave * kConvWords : nullptr;
            auto flush = [&](int k0, int mbase) {  // slots of steps k0 + mbase ..
                if (lane < kStage) {
                    const int oc = k0 + mbase + lane - (kLanes - 1);
                    if (oc >= 0 && oc < L) {
                        const Slot v = stg[lane];
                        if constexpr (LIN) {
                            bnd_h[oc] = v;
                        } else {
                            bnd_h[oc] = v.x;
                            bnd_f[oc] = v.y;
                        }
                    }
                }
            };
            auto block = [&](int bk) {
                const int k0 = bk * kLanes;
                // lane-0 conveyors for steps k0 .. k0+63 (column k = step); the
                // first chunk's row -1 is H = 0, F = 0 at the bias lane 0 reads
                // them with (see the hand-off below)
                {
                    const int col = k0 + lane;
                    in_res = in_res_nb;
                    in_res_nb = codes_at(col + kLanes);
                    const int bz = RI - 2 + (col % NB) + ((col % NB) == 0 ? NB : 0);
                    // (bz ge + zero) computed, not indexed: a lane-varying index
                    // into the argument table would copy the table to registers
                    in_bh = (!first && col < L) ? bnd_h[col] : C::pair_of(bz * a.gap_extend + C::zero_int(a));
                    in_bf = (!first && col < L) ? bnd_f[col] : C::pair_of((bz + 1) * a.gap_extend + C::zero_int(a));
                    if constexpr (CONV) {  // (the previous block's reads are done: one wave, in order)
                        cv[lane] = in_bh;
                        if constexpr (!LIN) cv[kLanes + lane] = in_bf;
                        cv[2 * kLanes + lane] = in_res;
                        cv[3 * kLanes + lane] = in_res_nb;
                    }
                }
                if (k0 == 0) {
#pragma unroll
                    for (int d = 0; d < PF; ++d) {
                        rcq[d] = shr1u(__builtin_amdgcn_readlane(in_res, d), d == 0 ? rc : rcq[d > 0 ? d - 1 : 0]);
                        read_words(rcq[d], W[d][0], W[d][1]);
                    }
                }
                // whole bias periods (steps past nsteps run pad columns: harmless)
                const int mend = min(kLanes, nsteps - k0);
                for (int m0 = 0; m0 < mend; m0 += NB) {
                    Slot* const sp = is_last_lane ? stg + (m0 % kStage) : scratch;
#pragma unroll
                    for (int b = 0; b < NB; ++b) {
                        const int m = m0 + b;
                        const uint32_t sbh = CONV ? cv[m] : __builtin_amdgcn_readlane(in_bh, m);
                        const uint32_t sbf = LIN ? 0u : CONV ? cv[kLanes + m] : __builtin_amdgcn_readlane(in_bf, m);
                        static_assert(NB % NBUF == 0, "buffer period");
                        Elem(&wa)[NQ] = W[b % NBUF][0];
                        Elem(&wb)[NQ] = W[b % NBUF][1];
                        rc = rcq[0];
#pragma unroll
                        for (int d = 0; d + 1 < PF; ++d) rcq[d] = rcq[d + 1];
                        // step b + PF's codes: lane 0 takes that column
                        // (the next block's first ones at the block's last steps)
                        const bool wrap = (b + PF >= NB) && (m0 + NB == kLanes);
                        const uint32_t sres_n =
                            CONV ? cv[2 * kLanes + m + PF]
                            : wrap ? __builtin_amdgcn_readlane(in_res_nb, (b + PF - NB) & (kLanes - 1))
                                   : __builtin_amdgcn_readlane(in_res, (m + PF) & (kLanes - 1));
                        rcq[PF - 1] = shr1u(sres_n, PF > 1 ? rcq[PF > 1 ? PF - 2 : 0] : rc);
                        read_words(rcq[PF - 1], W[(b + PF) % NBUF][0], W[(b + PF) % NBUF][1]);
                        // hand-off: the row above's bottom (H, F) from one step back
                        const V adj = diff(RI - 1 + (b == 0 ? NB : 0));
                        // affine: the row above's H is only row 0's next
                        // diagonal, so its (RI - 1) ge drop rides in the row-0
                        // profile words (staged with it) and only a rebase
                        // step's NB ge is subtracted here
                        const uint32_t up_raw = shr1u(sbh, hl);
                        const uint32_t up0 = LIN ? C::bits(C::from(up_raw) - adj)
                                                 : b == 0 ? C::bits(C::from(up_raw) - diff(NB))
                                                          : up_raw;
                        V f = LIN ? C::from(0u) : C::from(shr1u(sbf, fl)) - adj;
                        if (b == 0) {  // rebase: the bias period restarts
                            const V reb = diff(NB);
#pragma unroll
                            for (int r = 0; r < RI; ++r) {
                                H[r] = H[r] - reb;
                                if constexpr (!LIN) E[r] = E[r] - reb;
                            }
                            up_prev = C::bits(C::from(up_prev) - reb);
                        }
                        // H_diag + S for every row first (from the previous
                        // column's H), so H is then updated in place
                        V T[RI];
#pragma unroll
                        for (int r = 0; r < RI; ++r) {
                            const uint32_t ua = Img::word(wa, r), ub = Img::word(wb, r);
                            // low half: subject A's S for row r, high half: subject B's
                            const V sc = C::from(__builtin_amdgcn_perm(ub, ua, (r & 1) ? 0x07060302u : 0x05040100u));
                            T[r] = (r == 0 ? C::from(up_prev) : H[r - 1]) + sc;
                        }
                        // LIN: row 0's up term is the row above's bottom H (up0)
                        V up = C::from(up0);
                        up_prev = up0;
#pragma unroll
                        for (int r = 0; r < RI; ++r) {
                            V h;
                            if constexpr (LIN) {
                                h = C::max2(C::max3(H[r], up, T[r]), step(r + b));
                                up = h;
                            } else {
                                h = C::max3(E[r], f, T[r]);
                                const V mm = h - gog;
                                E[r] = C::max2(E[r], mm);
                                f = C::max3(f, mm, step(r + 1 + b));
                            }
                            V& ac = acc[r + b];
                            if (b & 1) {
                                if (r + 1 < RI) ac = C::max3(ac, h, H[r + 1]);  // H[r + 1]: cell (r + 1, step - 1)
                                else ac = C::max2(ac, h);
                            } else if (r == 0) {  // the even steps' other rows are partners above
                                ac = C::max2(ac, h);
                            }
                            H[r] = h;
                        }
                        hl = C::bits(H[RI - 1]);
                        if constexpr (!LIN) fl = C::bits(f);
                        // lane 63 finished column k - 63 (staged, see flush)
                        if constexpr (LIN) sp[b] = hl;
                        else sp[b] = make_uint2(hl, fl);
                        // pin the maxima at every step (left free, the compiler
                        // defers the reductions and keeps every h alive)
#pragma unroll
                        for (int q = 0; q < NACC; ++q) asm volatile("" : "+v"(acc[q]));
                    }
                    if (!last && ((m0 + NB) % kStage == 0 || m0 + NB >= mend))
                        flush(k0, (m0 + NB - 1) / kStage * kStage);
                }
            };
            for_blocks(nblk, block);
    };
    // stage rows [c0, c0 + CH) of codes 0..25 into image im as fp16 S + 2 ge
    // (the linear profile is biased by the gap, a.bias), threads [t0, ...)
    // in steps of `stride`
    auto stage = [&](Elem* im, int c0, int t0, int stride) {
        for (int t = t0; t < kCodes * NQ * kLanes; t += stride) {
            const int code = t / (NQ * kLanes);
            const int u = t % (NQ * kLanes);
            const int qq = u / kLanes, ln = u % kLanes;
            const int b = a.bias - 2 * a.gap_extend;
            im[t] = Img::load(prof16 + static_cast<size_t>(code) * a.prof_stride + c0 + ln * RI + Img::kRows * qq,
                              (!LIN && qq == 0) ? b + (RI - 1) * a.gap_extend : b, b);
        }
    };
    const int nch = (a.qpad + CH - 1) / CH;
    if constexpr (!PIPE) {
        for (int c0 = 0; c0 < a.qpad; c0 += CH) {
            __syncthreads();  // the previous chunk's LDS reads are done
            stage(img, c0, tid, kWavesPerWG * kLanes);
            __syncthreads();
            if (!hasA && !hasB) continue;  // wave-uniform; the barriers above are shared
            run_chunk(c0, img, c0 == 0, c0 + CH >= a.qpad, [](int nblk, auto& block) {
                for (int bk = 0; bk < nblk; ++bk) block(bk);
            });
        }
    } else {
        // PIPE: wave w runs chunk w (nch <= 4 chunks), each at its own pace:
        // it starts block bk (columns [64 bk, 64 bk + 64)) once wave w - 1 has
        // finished block bk + 1 (its lane 63 writes the boundary row of column
        // c at its step c + 63, i.e. in block (c + 63) / 64), told by a
        // progress count in LDS.  Wave w - 1 writes each column's boundary
        // value before wave w reads it, and wave w overwrites it (for wave
        // w + 1) only after reading it: one boundary array serves every
        // stage, and no wave ever waits for a later one.  (A workgroup barrier
        // per 64 steps instead tied every stage to the slowest SIMD's pace.)
        if (!hasA && !hasB) return false;  // workgroup-uniform (one pair per workgroup)
        Elem* mine = img + wave * (kCodes * NQ * kLanes);
        int* prog = reinterpret_cast<int*>(img + kWavesPerWG * (kCodes * NQ * kLanes));
        if (wave < nch) stage(mine, wave * CH, lane, kLanes);
        if (tid < kWavesPerWG) prog[tid] = 0;
        __syncthreads();
        if (wave < nch) {
            run_chunk(wave * CH, mine, wave == 0, wave == nch - 1, [&](int nb, auto& block) {
                for (int bk = 0; bk < nb; ++bk) {
                    if (wave > 0) {
                        const int need = min(bk + 2, nb);
                        // bounded: wave 0 never waits, so every stage progresses
                        for (int spin = 0; spin < (1 << 24); ++spin) {
                            if (__hip_atomic_load(prog + wave - 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >=
                                need)
                                break;
                            __builtin_amdgcn_s_sleep(1);
                        }
                    }
                    block(bk);
                    // this block's boundary stores before its progress count
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (lane == 0)
                        __hip_atomic_store(prog + wave, bk + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            });
        }
        __syncthreads();  // every stage done (and the images free)
    }
    // the lane's maximum (bias removed, offset kept: fp16 does not hold the
    // true scores above 2048 exactly), then the wave's
    V best = acc[0];
#pragma unroll
    for (int q = 1; q < NACC; ++q) best = C::max2(best, acc[q] - diff(q));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t o = static_cast<uint32_t>(__shfl_xor(static_cast<int>(C::bits(best)), off));
        best = C::max2(best, C::from(o));
    }
    if constexpr (PIPE) {
        // the stages' maxima (each covers its chunk's rows) to wave 0; the
        // images are free after the last round's barrier
        uint32_t* part = reinterpret_cast<uint32_t*>(img);
        if (wave < nch && lane == 0) part[wave] = C::bits(best);
        __syncthreads();
        if (wave != 0) return false;
        for (int w = 1; w < nch; ++w) best = C::max2(best, C::from(part[w]));
    }
    bool flagged = false;
    if (lane == 0) {
        const int ba = C::lo(best) - C::zero_int(a);
        const int bb = C::hi(best) - C::zero_int(a);
        if (hasA) {
            a.scores[a.subj_id[sa]] = ba;
            if (a.rescue_list && C::template flag<RI>(a, ba)) {
                list_publish(a.rescue_list, a.rescue_count, sa);
                flagged = true;
            }
        }
        if (hasB) {
            a.scores[a.subj_id[sb]] = bb;
            if (a.rescue_list && C::template flag<RI>(a, bb)) {
                list_publish(a.rescue_list, a.rescue_count, sb);
                flagged = true;
            }
        }
    }
    return __builtin_amdgcn_readfirstlane(flagged);
}

}  // namespace ix2
}  // namespace swk
