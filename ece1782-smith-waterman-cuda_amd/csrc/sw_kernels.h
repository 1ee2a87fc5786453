// sw_kernels.h — internal interface between the host driver (sw_capi.cpp)
// and the gfx950 kernels (sw_kernels.hip).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "sw_amd.h"  // sw_opts: the kernel-form overrides the shape choices below read

namespace swk {

// Record `msg` as this thread's sw_last_error() text and return `code`
// (sw_capi.cpp; used by the other host translation units, e.g. sw_group.cpp).
int set_error(int code, const std::string& msg);

constexpr int kLanes = 64;        // one database subject per lane (wave64)
constexpr int kGroupCols = 16;    // residue columns per packed group
constexpr int kGroupBytes = kLanes * kGroupCols;  // 1 KiB: [lane][16 residues]
constexpr int kProfileRows = 32;  // profile codes: 25 residues + PAD (25) + unused
constexpr int kPadCode = 25;      // residue code used for padding (scores 0)
// The byte a residue code is stored as in the device database (the profile
// rows follow it: row kStored[c] holds code c's scores).  The two-strips
// kernel reads its profile images with ds_read_b128 at 144 bytes (9 x 16)
// per code row; a 16-lane bank group spans 16 such slots, so stored bytes
// equal mod 16 share a slot with different addresses (one extra LDS cycle
// per group that holds both).  With 26 codes some pairs alias under any row
// stride; this order makes them rare ones: the six most frequent residues
// (L A G V E S) alone on slots 10-15, I beside the pad, K R D T P beside the
// codes a protein database does not hold (B J Z X *), and the eight rarest
// standard residues paired rarest with most frequent.  Modelled on C2's
// blocks (scripts/lds_conflict_model.py): 3.07 -> 1.48 extra LDS cycles per
// image read (the profiled launch measured 2.90 per LDS instruction with the
// alphabetical order).  The pad is stored as itself.
//                       A   R  N  D  C   Q  E   G   H   I  L   K  M   F  P  S   T  W   Y  V   B   J   Z   X   *   pad
constexpr uint8_t kStored[26] = {11, 1, 5, 2, 22, 6, 14, 12, 23, 9, 10, 0, 24, 7, 4, 15, 3, 21, 8, 13, 16, 17, 18, 19, 20, 25};
// ... and its inverse: the code a stored byte stands for
constexpr uint8_t kCodeOf[26] = {11, 1, 3, 16, 14, 2, 5, 13, 18, 9, 10, 0, 7, 19, 6, 15, 20, 21, 22, 23, 24, 17, 4, 8, 12, 25};
constexpr int kWavesPerWG = 4;
// f16_step entries the intra kernels read (IntraArgs): up to RI + the bias
// period (intra_period) + 1
constexpr int kIntraSteps = 40;

// Shared by the inter kernels: one wave's residues for SG columns.
template <int SG>
struct Residues {
    uint32_t w[SG / 4];
    __device__ __forceinline__ void load(const uint8_t* p) {
        if constexpr (SG == 16) {
            const int4 v = *reinterpret_cast<const int4*>(p);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        } else if constexpr (SG == 8) {
            const int2 v = *reinterpret_cast<const int2*>(p);
            w[0] = v.x; w[1] = v.y;
        } else {
            w[0] = *reinterpret_cast<const uint32_t*>(p);
        }
    }
    __device__ __forceinline__ uint32_t code(int jj) const { return (w[jj >> 2] >> (8 * (jj & 3))) & 0xffu; }
};

// Packed database, inter-sequence part (the layout
// replaces the reference's [block][col][32-lane] short interleave,
// SWSolver.cu:316):
//   residues : for block b, at byte blk_off[b]: ngroups[b] groups, each
//              [64 lanes][16 residue codes]  (one dwordx4 per lane)
//   bnd_h/f  : int32 boundary rows in the SAME index space as residues
//              (4 bytes per residue byte), the DP row handed from one
//              query strip to the next (replaces the 3.7 GB short
//              "collapsed" matrix, SWSolver.cu:231-258,288)
struct InterArgs {
    const uint8_t* residues;
    const uint64_t* blk_off;     // byte offset of group 0 of each block
    const uint32_t* blk_groups;  // number of 16-column groups per block
    // the single-wave fp16/int16 kernel's block widths: the longest subject
    // rounded up to 8 columns, not 16 (nullable: groups x 16)
    const uint32_t* blk_cols;
    const int32_t* lane_ids;     // [nblocks][64] result slot, -1 = empty lane
    int32_t nblocks;
    const int8_t* prof;          // [kProfileRows][prof_stride] query profile (see host)
    int32_t prof_stride;         // bytes per profile row (>= qpad, multiple of 16)
    int32_t qpad;                // query length rounded up to the strip height
    int32_t gap_open;
    int32_t gap_extend;
    int32_t* bnd_h;
    int32_t* bnd_f;
    int32_t* scores;             // scores[id]
    // int16 kernel: blocks with a lane near int16 saturation are appended
    // here (count at rescue_count) and re-scored by the int32 kernel, which
    // in list mode (blk_list != nullptr) walks only the listed blocks.
    int32_t* rescue_list;
    int32_t* rescue_count;
    const int32_t* blk_list;
    const int32_t* blk_count;
    // blocks [0, blk_first) are handled by the cooperative kernel; the
    // one-block-per-wave kernels start at blk_first
    int32_t blk_first;
    // fp16 kernel: a lane whose running maximum reaches this flags its block
    int32_t sat_limit;
    // fp16 kernel, biased cell (sw_inter_x2.hip): f16_step[j] = the packed
    // fp16 pair (j * gap_extend + f16 offset), j = 0..31, and f16_gog =
    // packed (gap_open - gap_extend); host-built so they stay in SGPRs
    // All fp16 cell values carry the offset f16_zero = (z, z), z = -2048 +
    // 2 ge: fp16 holds every integer in [-2048, 2048] exactly, so the
    // shifted cell is exact for true values up to ~4096 (max/add commute
    // with the shift; sw_capi.cpp states the bound).  f16_step[j] is then
    // the pair (j ge + z), and f16_diff the unshifted pairs (4 ge, 8 ge,
    // 16 ge): the rebase per sub-group of 4 or 8 columns, the row-group reset.
    uint32_t f16_step[32];
    uint32_t f16_gog;
    uint32_t f16_zero;
    uint32_t f16_diff[3];
    // sw_inter_x2p: its pair blocks are [blk_base, blk_first) (merged) or
    // [blk_base, nblocks); blocks below blk_base run elsewhere
    int32_t blk_base;
    // sw_scan_lpt: blocks [blk_base, blk_quad) run by wave quads, or (affine
    // gaps, blk_tri != 0) by 3-wave groups whose workgroup's fourth wave runs
    // a single-wave block
    int32_t blk_quad;
    int32_t blk_tri;
    // sw_scan_lpt: blocks [blk_tail, nblocks) (the narrowest) run by wave
    // pairs after the single-wave range (0 or nblocks: none)
    int32_t blk_tail;
    // fp16 kernels: the largest flagged block id (atomicMax; nullable), read
    // back by the host to route the widest blocks to int16 next time
    int32_t* rescue_max;
    // per-block timeline (builds with -DSW_TRACE_BLOCKS only; env
    // SW_TRACE_FILE): [block][start, end, HW_ID, XCC_ID | kind << 32],
    // s_memrealtime (100 MHz) stamps, host-mapped memory
    uint64_t* trace;
};

// Long subjects: one wave per subject, query rows spread over the 64 lanes,
// anti-diagonal wavefront with wave_shr DPP hand-off between lanes.
struct IntraArgs {
    const uint8_t* residues;     // plain concatenated codes of the long subjects
    const uint64_t* subj_off;    // byte offset of each long subject
    const int32_t* subj_len;
    const int32_t* subj_id;
    int32_t nsubj;
    const int8_t* prof;          // [chunk][kProfileRows][64 lanes][RIP] (host-built)
    int32_t qpad;                // multiple of 64 * rows-per-lane
    int32_t gap_open;
    int32_t gap_extend;
    int32_t* bnd_h;              // per subject: subj_off-indexed int32 rows
    int32_t* bnd_f;
    int32_t* scores;
    // sw_intra_x2 (packed fp16): the int16 profile [kProfileRows][prof_stride]
    // in `prof`, minus `bias` (the linear profile's gap bias) = raw S
    int32_t prof_stride = 0;
    int32_t bias = 0;
    int32_t sat_limit = 0;       // flag subjects whose maximum reaches this
    uint32_t f16_step[kIntraSteps] = {};  // as InterArgs (j ge + z, j ge + z), j < RI + period
    uint32_t f16_zero = 0;       // the offset z = -2048 + 2 ge of every fp16 cell value
    uint32_t f16_gog = 0;        // packed fp16 (go - ge, go - ge)
    int32_t* rescue_list = nullptr;
    int32_t* rescue_count = nullptr;
    // sw_intra in list mode: only subjects subj_list[0 .. *list_count)
    const int32_t* subj_list = nullptr;
    const int32_t* list_count = nullptr;
    // sw_scan_lpt: pairs [0, pipe_pairs) run in the pipelined form; the
    // launch's ordinary intra workgroups skip them
    int32_t pipe_pairs = 0;
    // ... and pairs [pipe_tail, ...) too (the launch's last items: the
    // shortest long subjects, whose latency the pipeline cuts at the end)
    int32_t pipe_tail = 0x7fffffff;
};

// ---- device-side rescue lists: [count, item 0, item 1, ...] --------------
// A 16-bit kernel appends the blocks / subjects whose values may have left
// its exact range; the next stage re-scores them.  Entries past the count
// hold -1: whoever takes an entry resets it, so every list is all -1 past
// its count when a scan starts (the host fills new lists with -1 and zeroes
// the counts per scan), and a consumer running in the SAME launch as the
// producer (sw_scan_lpt's drain) can wait for an entry whose slot a
// producer has claimed but not yet written.
#if defined(__HIPCC__)
// threadIdx.x made opaque at each read: the merged launch's looped form runs
// every scan form inside one loop, and the compiler hoists what the forms
// derive from the thread index (lane and LDS addresses) out of it, holding
// all of them live across every form at once (sw_inter_x2.hip sw_scan_lpt).
// Read through this, each form derives them anew per entry.
__device__ __forceinline__ int tid_x() {
    int t = static_cast<int>(threadIdx.x);
    asm volatile("" : "+v"(t));
    return t;
}
// Producer: this wave's results (its scores, its boundary rows) are made
// visible device-wide before the entry, so a re-scoring stage on another XCD
// overwrites them, not the reverse.
__device__ __forceinline__ void list_publish(int32_t* items, int32_t* count, int32_t item) {
    __threadfence();
    const int slot = atomicAdd(count, 1);
    __hip_atomic_store(items + slot, item, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Consumer in a later launch (the entry is written): read entry i, reset it.
// Wave-uniform.
__device__ __forceinline__ int32_t list_take(const int32_t* items, int i) {
    int32_t* p = const_cast<int32_t*>(items) + i;
    const int32_t v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    __hip_atomic_store(p, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v;
}
// Consumer in the producer's launch: wait until entry i is written, then
// reset it.  The producer stores the entry right after its atomicAdd and a
// wave is not preempted, so the entry appears within microseconds; the wait
// is still bounded (`bound` polls, by default 2^22: about 0.1 s) so a wave can
// never hang here, and a timeout is not silent: it sets *fault (host-visible,
// mapped), the library fails the next call on that handle (SW_E_DEVICE) and
// the caller skips the entry.  (sw_opts drain_spin 0, tests: every wait times
// out at once.)
__device__ __forceinline__ int32_t list_wait_take(int32_t* items, int i, int32_t* fault, int32_t bound) {
    int32_t* p = items + i;
    int32_t v = -1;
    for (int spin = 0; spin < bound; ++spin) {
        v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v >= 0) break;
        __builtin_amdgcn_s_sleep(1);
    }
    if (v >= 0)
        __hip_atomic_store(p, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (fault)
        __hip_atomic_store(fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return v;
}
// Claim up to `want` entries [start, start + n) past the list's head; 0 when
// none are left (or other workgroups keep winning: they drain the rest).
__device__ __forceinline__ int list_claim(int32_t* count, int32_t* head, int want, int* start) {
    int h = __hip_atomic_load(head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int tries = 0; tries < 256; ++tries) {
        const int c = __hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (h >= c) return 0;
        const int nh = h + want < c ? h + want : c;
        if (__hip_atomic_compare_exchange_strong(head, &h, nh, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
            *start = h;
            return nh - h;
        }
    }
    return 0;
}
#endif

// Shape of the inter kernel for this gap model: R query rows per strip x SG
// columns per software-pipelined sub-group; x2s: the packed two-strips
// kernel (int16 profile), f16: its fp16 form.  x2_ok: 2 = the scan is
// provably int16-safe (any packed kernel may run); 1 = a guarded packed
// kernel may run (saturating blocks are re-scored at int32); 0 = int32 only.
// o.int16_guard / o.inter_variant override the choice (tests, A/B).
struct InterShape {
    int R, SG;
    bool x2s = false;
    bool f16 = false;
};
InterShape inter_shape(bool affine, int x2_ok, const sw_opts& o);
// true if the chosen inter kernel may flag blocks for int32 re-scoring
// (16-bit kernels beyond the static int16 bound).
inline bool inter_needs_rescue(const InterShape& v, int x2_ok) { return v.f16 || (v.x2s && x2_ok != 2); }
// true if the chosen inter kernel has a wave-pair form (two-strips 32x8).
inline bool inter_has_pair(const InterShape& v) { return v.x2s && v.R == 64 && v.SG == 8; }
// Wide-block cut-off for the cooperative kernel: residues / divisor columns
// (0 = the chosen inter kernel does not use it: one subject per lane with two
// strips per pass has no long single-wave tail, coop on/off within 1 %).
inline int inter_coop_divisor(const InterShape& v) { return v.x2s ? 0 : 530000; }
// Name of the per-wave inter kernel launch_inter() runs, e.g. "sw_inter_x2s<32,8,affine,fp16>".
const char* inter_kernel_name(const InterShape& v, bool affine);
// Query rows per lane the intra kernel uses for this query (2..16, even).
int intra_rows_for(int qlen, int longest);
// Bytes of one intra profile chunk (64*ri query rows, 32 codes).
int intra_chunk_bytes(int ri);
__host__ __device__ constexpr int intra_rip(int RI) { return (RI + 3) / 4 * 4; }

hipError_t launch_inter(const InterArgs& a, bool affine, const InterShape& v, hipStream_t s);
// Wide blocks [0, ncoop): one 4-wave workgroup per block, the waves pipelined
// over query strips (skew: strip k+1 one sub-group behind strip k).
hipError_t launch_inter_coop(const InterArgs& a, int ncoop, bool affine, bool skew, hipStream_t s);
int inter_coop_rows();
// One subject per lane, two R-row query strips per pass in the two int16
// halves (sw_inter_x2.hip); qpad is a multiple of 2R; boundary rows are
// (H | F << 16) dwords in bnd_h.
hipError_t launch_inter_x2s(const InterArgs& a, int R, int SG, bool affine, bool f16, hipStream_t s);
// The int16 packed kernel in list mode (blk_list / blk_count set): the
// second stage of the fp16 rescue chain.
hipError_t launch_inter_x2s_list(const InterArgs& a, bool affine, hipStream_t s);
// Wave groups over the widest blocks of a two-strips 32x8 scan
// (sw_inter_x2p; group = 2: pairs, 4: quads): same results as
// launch_inter_x2s, 1/group of the block latency.  merged: one launch, blocks
// [blk_base, blk_first) by groups, [blk_first, nblocks) one per wave;
// otherwise blocks [blk_base, nblocks) by groups only.
hipError_t launch_inter_x2p(const InterArgs& a, bool affine, bool f16, bool merged, int group, hipStream_t s);
// One launch for the whole fp16 scan, longest work first (sw_scan_lpt):
// order[0..n) names each workgroup's work, >= 0 an inter workgroup (a as for
// launch_inter_x2p merged, with blocks [blk_base, blk_quad) by quads, then
// [blk_quad, blk_first) by pairs), < 0 intra workgroup -1 - order[k] (ia as
// for launch_intra_x2: 4 subject pairs per workgroup).  Intra rows per lane
// 4, 6 or 8.
// drain (nullable, DEVICE memory): the launch also re-scores what its fp16
// cells flag — each workgroup, after its own work, takes entries of the four
// rescue lists until none are left: int16 subject pairs of list 1 (i16: the
// int16 intra form, flagging into list 2), int16 blocks of list A (a16: the
// x2s list form, flagging into list B), int32 subjects of list 2 (i32:
// sw_intra's body, rows per lane = ri) and int32 blocks of list B (a32:
// sw_inter's body) — the four rescue launches that otherwise follow the scan
// (and their ~5 us each of command-processor time).  The stages use their own
// boundary rows (the deferred tails' rows).  In device memory, not in the
// kernel arguments: read from kernel arguments, the compiler kept the drain's
// values in registers across the scan loops and spilled.
struct DrainArgs {
    InterArgs a16;
    InterArgs a32;
    IntraArgs i16;
    IntraArgs i32;
    int32_t* lists[4];  // list A, B, 1, 2: [count, items...]
    int32_t* heads[4];  // their dequeue heads (zeroed per scan)
    int32_t* fault;     // host-mapped word: a claimed entry never appeared (list_wait_take)
    int32_t spin;       // list_wait_take's bound (sw_opts drain_spin)
};
bool lpt_supported(int ri);
// next (nullable; zero at launch): with it, a table of at least 3 rounds of
// resident workgroups runs one workgroup per resident slot, each taking its
// next entry of order[] from this counter when it has finished one (the
// dispatcher's per-workgroup gaps avoided); otherwise one workgroup per
// entry.  loop_grid > 0 (tests): that form with that many workgroups.
// rows: query rows per pass, 64 (32-row strips) or, linear gaps only, 96.
// cus: the device's compute units (the looped grid's size).
hipError_t launch_scan_lpt(const InterArgs& a, const IntraArgs& ia, const int32_t* order, int n, bool affine, int ri, int cus,
                           hipStream_t s, const DrainArgs* drain = nullptr, int32_t* next = nullptr,
                           int loop_grid = 0, int rows = 64);
// Lanes whose 16-bit running maximum reaches this may have overflowed.
constexpr int kSat16 = 32767 - 1152;
// The two-subjects intra kernel's widest shape: 20 rows per lane, in the
// same 4-wave workgroups: the 26-code image of 1,280 rows (66.5 KB) leaves two
// workgroups per CU, 2 waves per SIMD.  (Measured on C5: 6-wave workgroups did
// not fit two per CU, 2 + 2 + 1 + 1 waves per SIMD each: 5,550 GCUPS; 12-wave
// ones, one per CU, left whole CUs idle in the last round: 7,475; 4-wave:
// 8,892.)
constexpr int kIntraX2MaxRI = 20;
// Steps per bias period of the intra kernel at RI rows per lane (one rebase
// of every row's H and E per period): 16 at the widest shape, whose 2 waves
// per SIMD leave registers for the 8 more anti-diagonal maxima; 8 otherwise.
// (8 at RI 20 too: C5 8,809 against 8,983 GCUPS, profiles/r05_ab/intra_period16/)
constexpr int intra_period(int ri) { return ri == kIntraX2MaxRI ? 16 : 8; }
// Its biased cell stores values up to this many gap extensions above the
// true ones (row RI - 1 at the last step of a bias period, + 2 ge in the
// profile, + the F floor's step).
constexpr int intra_bias_rows(int ri) { return ri + intra_period(ri) + 2 > 26 ? ri + intra_period(ri) + 2 : 26; }

// int32 re-scoring of the blocks a 16-bit kernel listed (device-side count);
// strips of rescue_rows(affine) query rows.
int rescue_rows(bool affine);
hipError_t launch_inter_rescue(const InterArgs& a, bool affine, hipStream_t s);
hipError_t launch_intra(const IntraArgs& a, int ri, bool affine, hipStream_t s);
// Two subjects per wave, packed fp16 (sw_intra_x2.hip); rows per lane 4..16,
// and 20 when intra_x2_rows_for allows it.
hipError_t launch_intra_x2(const IntraArgs& a, int ri, hipStream_t s);
// its int16 form over the device-side list a.subj_list / a.list_count
hipError_t launch_intra_x2_list16(const IntraArgs& a, int ri, hipStream_t s);
// ... and over every subject (the chain's first stage when fp16 would flag most)
hipError_t launch_intra_x2_int16(const IntraArgs& a, int ri, hipStream_t s);
// wide: 0 = rows per lane 4..16; 1 = 20 too when forced (sw_opts
// intra_x2_rows, > 0: a forced shape); 2 = 20 by the cost model too.  The host allows 20 only
// where no merged launch can take the scan (no inter blocks) and the fp16
// bias of row 19 fits, and picks it only for affine gaps (the linear cell
// lost 35 % at 20 on C5: its cheaper steps need the third wave per SIMD).
int intra_x2_rows_for(int qlen, int longest, int wide, int forced);

// Traceback of chosen hits (sw_align.hip): cpu.cpp's tie rules for a linear
// gap (gap == gap_extend), this build's extension of them for affine gaps.
struct AlignArgs {
    const uint8_t* query;
    int32_t qlen;
    const uint8_t* subj;       // the hits' subject residues, concatenated
    const int64_t* subj_off;   // n+1 offsets
    int32_t n;
    const int8_t* mat;         // 25 x 25
    int32_t gap;               // gap open (a 1-residue gap)
    int32_t gap_extend;        // each further residue (== gap: linear)
    uint8_t* dirs;             // per hit: (qlen + slen + 1) x (qlen + 1) direction bytes
    const int64_t* dirs_off;   // per hit offset into dirs
    int32_t* hbuf;             // per hit: 3 x (qlen + 1) int32 diagonal scratch for linear gaps, 7 x (qlen + 1) when gap_extend != gap (sw_align_affine: H x3, E x2, F x2)
    int32_t* out;              // per hit: score, q_begin, q_end, s_begin, s_end, ops_len
    char* ops;                 // per hit: ops_stride bytes (may be null)
    int64_t ops_stride;
};
hipError_t launch_align(const AlignArgs& a, hipStream_t s);

// Synthetic databases generated on the device (sw_synth.hip).
struct SynthFill {
    uint8_t* res;                // packed inter residues (layout of InterArgs)
    const uint64_t* blk_off;
    const uint32_t* blk_groups;
    const int32_t* lane_local;   // [nblocks][64] local subject id, -1 = empty
    const int32_t* lane_len;     // [nblocks][64] subject length
    int64_t nblocks;
    uint8_t* lres;               // intra residues (IntraArgs layout)
    const uint64_t* loff;
    const int32_t* llen;
    const int32_t* lid;          // local ids
    int32_t nlong;
    uint64_t seed;
    int64_t id_base;             // global id = id_base + local id
    const uint8_t* lut;          // [65536] uniform u16 -> residue code
};
hipError_t launch_synth_fill(const SynthFill& f, hipStream_t s);
uint64_t synth_hash(uint64_t seed, uint64_t id, uint64_t k);

// Query profiles built on the device (sw_profile.hip) from the query codes
// and the matrix in the kernel arguments: rows [row0, row1) per launch (at
// most kProfQueryChunk), q[] = the codes of rows [row0, min(row1, qlen)).
//   p8  : [kProfileRows][stride] int8, S + bias (rows >= qlen, codes >= 25: bias)
//   p16 : the same values as int16 (null: not built)
//   pin : the int32 intra kernel's lane-slotted image, rows < qpad_intra:
//         [chunk of 64 ri rows][code][lane][rip] (null: not built)
// The first launch also zeroes the rescue lists' counters and dequeue heads
// (reset[2] := -1, the largest-flagged-block slot; null pointers skipped).
constexpr int kAlphabet = 25;
constexpr int kProfQueryChunk = 2048;
struct ProfileArgs {
    int8_t* p8;
    int16_t* p16;
    int8_t* pin;
    int32_t stride;
    int32_t qlen;
    int32_t row0, row1;
    int32_t bias;
    int32_t ri, rip, qpad_intra;
    int32_t* reset[10];
    int8_t mat[kAlphabet * kAlphabet + 15];
    uint8_t q[kProfQueryChunk];
};
hipError_t launch_build_profile(const ProfileArgs& a, hipStream_t s);

// A ranking input (sw_rank.h topk_key): entry g of [0, n) is keys[g], or the
// key of (scores[r], gid ? gid[r] : id_base + r) with r = rid ? rid[g] : g —
// rid: a database's result ids (sw_scan_topk: only mapped slots), gid: a
// shard's global ids (sw_topk_device_ids).
struct TopkSrc {
    const int32_t* scores;
    const int64_t* keys;
    const int32_t* rid;
    const int32_t* gid;
    int64_t id_base;
};
// Device top-K (sw_topk.hip): keys = score << 32 | (2^31 - 1 - id), best
// first, of entries [0, n) of src.  The workspace holds the stages' keys and,
// at its start, the one-launch form's counter (zero between launches: the
// launch that uses it resets it).
size_t topk_workspace_bytes(int64_t n, int k);
hipError_t launch_topk(const TopkSrc& src, int64_t n, int k, int64_t* out, int64_t* work, hipStream_t s);

}  // namespace swk
