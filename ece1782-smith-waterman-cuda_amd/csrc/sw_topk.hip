// sw_topk.hip — device top-K of a score vector, for the multi-GPU exchange
// (each rank's best K (score, id) go to one RCCL all-gather).
//
// The radix select (sw_rank.h) in stages: a workgroup holds a chunk of keys
// in registers (16 per thread: 4,096 keys for 256 threads, 16,384 for 1,024)
// and writes its chunk's k best; the stage repeats on the survivors (chunks x
// k keys) until one chunk remains, whose workgroup also sorts its k keys
// (bitonic in LDS).  No host synchronisation: every stage's size is known
// from n and k.  A scan that runs as the merged launch ranks its scores in
// that launch's tail instead (sw_rank.h rank_tail, sw_scan_lpt).
//
// Workgroup size: a ranking launched beside a scan waits for CUs: the scan's
// workgroups hold every CU with 2 waves per SIMD at 256 VGPRs each.  A
// 1,024-thread workgroup (4 waves per SIMD at 66 VGPRs, 72 with the
// allocation granule) fits nowhere until the scan's grid has drained: its
// kernel traces showed the ranking's first stage taking a whole scan (6.15 ms
// on C2).  For k <= 1,024 the stages run 256-thread workgroups (one wave per
// SIMD), which fit in the registers one finished scan workgroup leaves:
// C2 (570k scores, k = 100) ranks in 3 launches (140 chunks, 4, 1); larger k
// keeps 1,024 threads (a stage must keep fewer keys than it reads).
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

static int64_t topk_chunk(int k) { return (k <= kTopkSmallK ? 256 : 1024) * kTopkPer; }

// Workspace bytes sw_topk_device needs for n inputs and k outputs.
size_t topk_workspace_bytes(int64_t n, int k) {
    size_t total = 0;
    int64_t cur = n;
    const int64_t chunk = topk_chunk(k);
    while (cur > chunk) {
        const int64_t chunks = (cur + chunk - 1) / chunk;
        cur = chunks * k;
        total += static_cast<size_t>(cur) * sizeof(int64_t);
    }
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
    return k <= kTopkSmallK ? launch_topk_t<256>(src, n, k, out, work, s)
                            : launch_topk_t<1024>(src, n, k, out, work, s);
}

}  // namespace swk
