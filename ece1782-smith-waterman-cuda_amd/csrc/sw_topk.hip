// sw_topk.hip — device top-K of a score vector, for the multi-GPU exchange
// (each rank's best K (score, id) go to one RCCL all-gather).
//
// The radix select (sw_rank.h): a workgroup holds a chunk of keys in
// registers and writes its chunk's k best; a last selection over the chunks'
// survivors, sorted (bitonic in LDS), is the result.  No host
// synchronisation: every size is known from n and k.
//
// One launch (sw_topk_fused) whenever k <= 1,024 and the chunks' survivors
// fit one workgroup's final selection (C2: 570k scores, k = 100, 70 chunks of
// 8,192): its workgroups arrive on a counter after writing their survivors
// and the last to arrive ranks them.  The ranking runs on the exchange
// stream beside the next scan, and only a launch that starts in the gap
// before the next scan's grid fills the CUs runs at once: round 4's chained
// stages (C2: 140 chunks -> 4 -> 1) left their later launches queued behind
// the next scan (C2's second stage 953 us on average, the 1/8 share's final
// 592 us; their first stage 16 us: profiles/r05_ab/rank_in_tail/*sep*).
// Ranking inside the scan's merged launch instead (the last workgroups to
// finish, d018fbd) cost the launch 58 us on C2 and 43 us on the 1/8 share.
// Larger k keeps the chained stages (16 keys per thread: 4,096-key chunks for
// 256 threads, 16,384 for 1,024).
//
// Workgroup size: a ranking launched beside a scan waits for CUs: the scan's
// workgroups hold every CU with 2 waves per SIMD at 256 VGPRs each.  A
// 1,024-thread workgroup (4 waves per SIMD at 66 VGPRs, 72 with the
// allocation granule) fits nowhere until the scan's grid has drained: its
// kernel traces showed the ranking's first stage taking a whole scan (6.15 ms
// on C2).  For k <= 1,024 the stages run 256-thread workgroups (one wave per
// SIMD), which fit in the registers one finished scan workgroup leaves
// (chained, C2's 570k scores at k = 100 took 3 launches: 140 chunks, 4, 1);
// larger k keeps 1,024 threads (a stage must keep fewer keys than it reads).
#include <algorithm>

#include "sw_rank.h"

namespace swk {

constexpr int kTopkPer = 16;       // keys per thread
constexpr int kTopkSmallK = 1024;  // k up to this: 256-thread workgroups (4,096-key chunks)

// Keys [blockIdx.x chunk] of src (first stage) or of the previous stage's
// output (src.keys); FINAL: one workgroup, sorted output.
template <int kTopkThreads, bool FINAL>
__global__ __launch_bounds__(kTopkThreads) void sw_topk_select(TopkSrc src, int64_t n, int k,
                                                              int64_t* __restrict__ out) {
    __shared__ TopkLds<kTopkThreads> L;
    __shared__ int64_t sorted[FINAL ? kTopkMaxK : 1];
    constexpr int kTopkChunk = kTopkThreads * kTopkPer;  // keys per workgroup
    const int t = threadIdx.x;
    const int64_t start = static_cast<int64_t>(blockIdx.x) * kTopkChunk;
    const int m = static_cast<int>(min(static_cast<int64_t>(kTopkChunk), n - start));  // keys in this chunk
    uint64_t u[kTopkPer];
#pragma unroll
    for (int j = 0; j < kTopkPer; ++j) {
        const int i = j * kTopkThreads + t;
        u[j] = i < m ? topk_key(src, start + i) : 0;
    }
    if constexpr (FINAL) {
        topk_select<kTopkThreads>(u, m, k, L, [&](int pos, uint64_t v) { sorted[pos] = key_of(v); });
        topk_sort_out<kTopkThreads>(sorted, min(m, k), k, out);
    } else {
        int64_t* const o = out + static_cast<int64_t>(blockIdx.x) * k;
        topk_select<kTopkThreads>(u, m, k, L, [&](int pos, uint64_t v) { o[pos] = key_of(v); });
        for (int i = min(m, k) + t; i < k; i += kTopkThreads) o[i] = kKeyPad;
    }
}

// The one-launch form: chunks of at most 8,192 keys (32 per thread), at
// least 4,096 keys each up to 64 chunks; the final selection holds the
// chunks' k survivors each in the same 8,192.
constexpr int kFusedPer = 32;
constexpr int kFusedMaxK = 1024;
constexpr int64_t kFusedCap = 256 * kFusedPer;
struct TopkFused {
    TopkSrc src;
    int64_t n;
    int32_t k, nchunks, chunk;
    int64_t* work;  // nchunks x k survivors
    int64_t* out;
    int32_t* ctl;   // arrivals (zero between launches)
};

static bool fused_plan(int64_t n, int k, TopkFused* r) {
    if (k > kFusedMaxK || n <= 0) return false;
    int64_t c = std::max<int64_t>((n + kFusedCap - 1) / kFusedCap, std::min<int64_t>(64, (n + 4095) / 4096));
    const int64_t ch = (n + c - 1) / c;
    c = (n + ch - 1) / ch;
    if (c > 1 && c * k > kFusedCap) return false;
    r->n = n;
    r->k = k;
    r->nchunks = static_cast<int32_t>(c);
    r->chunk = static_cast<int32_t>(ch);
    return true;
}

// Chunk blockIdx.x's k best to r.work (write-through 8-byte stores), then
// one arrival per workgroup after every wave's stores have completed; the
// last to arrive reads the survivors with sc1 loads (the hand-off form
// MI355X_MICROARCH.md measures valid without a release fence, whose L2
// write-back would also flush the concurrent scan's dirty lines), selects
// and sorts the k best and resets the counter.  One chunk: select and sort.
//
// What the hand-off relies on: on gfx94x / gfx950 (CDNA3/4)
// (1) an agent-scope relaxed store is a write-through (sc1) store that
// reaches the L2 every CU of the agent reads, and an agent-scope relaxed load
// bypasses the CU's L1 (sc1), and (2) vector-memory STORES are counted in
// vmcnt (these targets have no separate vscnt counter, unlike gfx10+), so
// `s_waitcnt vmcnt(0)` in every wave, then the barrier, completes the
// workgroup's stores before its arrival is counted.  Targets without both
// would need a release / acquire pair (or the chained stages): the build
// refuses them rather than rank on stale survivors.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__)
#error "sw_topk_fused: the write-through hand-off is specified for gfx942 / gfx950 only"
#endif
__global__ __launch_bounds__(256) void sw_topk_fused(TopkFused r) {
    constexpr int T = 256;
    __shared__ TopkLds<T> L;
    __shared__ int64_t sorted[kFusedMaxK];
    __shared__ int last;
    const int t = threadIdx.x;
    const int64_t start = static_cast<int64_t>(blockIdx.x) * r.chunk;
    const int m = static_cast<int>(min(static_cast<int64_t>(r.chunk), r.n - start));
    uint64_t u[kFusedPer];
#pragma unroll
    for (int j = 0; j < kFusedPer; ++j) u[j] = j * T + t < m ? topk_key(r.src, start + j * T + t) : 0;
    if (r.nchunks == 1) {
        topk_select<T>(u, m, r.k, L, [&](int pos, uint64_t v) { sorted[pos] = key_of(v); });
        topk_sort_out<T>(sorted, min(m, r.k), r.k, r.out);
        return;
    }
    int64_t* const w = r.work + static_cast<int64_t>(blockIdx.x) * r.k;
    topk_select<T>(u, m, r.k, L, [&](int pos, uint64_t v) {
        __hip_atomic_store(w + pos, key_of(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    });
    for (int i = min(m, r.k) + t; i < r.k; i += T)
        __hip_atomic_store(w + i, kKeyPad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) last = __hip_atomic_fetch_add(r.ctl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == r.nchunks - 1;
    __syncthreads();
    if (!last) return;  // workgroup-uniform
    const int mf = r.nchunks * r.k;
#pragma unroll
    for (int j = 0; j < kFusedPer; ++j)
        u[j] = j * T + t < mf ? key_ord(__hip_atomic_load(r.work + j * T + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                              : 0;
    topk_select<T>(u, mf, r.k, L, [&](int pos, uint64_t v) { sorted[pos] = key_of(v); });
    topk_sort_out<T>(sorted, min(mf, r.k), r.k, r.out);
    if (t == 0) __hip_atomic_store(r.ctl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the next launch's
}

static int64_t topk_chunk(int k) { return (k <= kTopkSmallK ? 256 : 1024) * kTopkPer; }

// Workspace bytes sw_topk_device needs for n inputs and k outputs: the
// counter's 256 bytes, then the chained stages' keys (or the one launch's).
size_t topk_workspace_bytes(int64_t n, int k) {
    size_t total = 0;
    int64_t cur = n;
    const int64_t chunk = topk_chunk(k);
    while (cur > chunk) {
        const int64_t chunks = (cur + chunk - 1) / chunk;
        cur = chunks * k;
        total += static_cast<size_t>(cur) * sizeof(int64_t);
    }
    TopkFused f{};
    if (fused_plan(n, k, &f)) total = std::max(total, static_cast<size_t>(f.nchunks) * k * sizeof(int64_t));
    return total + 256;
}

template <int T>
static hipError_t launch_topk_t(const TopkSrc& src0, int64_t n, int k, int64_t* out, int64_t* work, hipStream_t s) {
    constexpr int64_t chunk = T * kTopkPer;
    TopkSrc src = src0;
    int64_t cur = n;
    int64_t* w = work;
    while (cur > chunk) {  // each stage keeps k of every chunk's keys (k <= chunk / 4)
        const int64_t chunks = (cur + chunk - 1) / chunk;
        hipLaunchKernelGGL((sw_topk_select<T, false>), dim3(static_cast<unsigned>(chunks)), dim3(T), 0, s, src, cur,
                           k, w);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        src = TopkSrc{};
        src.keys = w;
        cur = chunks * k;
        w += cur;
    }
    hipLaunchKernelGGL((sw_topk_select<T, true>), dim3(1), dim3(T), 0, s, src, cur, k, out);
    return hipGetLastError();
}

hipError_t launch_topk(const TopkSrc& src, int64_t n, int k, int64_t* out, int64_t* work, hipStream_t s) {
    if (k <= 0 || k > kTopkMaxK || (!src.keys && !src.scores && n > 0)) return hipErrorInvalidValue;
    int64_t* const keys = work + 256 / sizeof(int64_t);  // after the counter
    TopkFused f{};
    if (fused_plan(n, k, &f)) {
        f.src = src;
        f.work = keys;
        f.out = out;
        f.ctl = reinterpret_cast<int32_t*>(work);
        hipLaunchKernelGGL(sw_topk_fused, dim3(static_cast<unsigned>(f.nchunks)), dim3(256), 0, s, f);
        return hipGetLastError();
    }
    return k <= kTopkSmallK ? launch_topk_t<256>(src, n, k, out, keys, s)
                            : launch_topk_t<1024>(src, n, k, out, keys, s);
}

}  // namespace swk
