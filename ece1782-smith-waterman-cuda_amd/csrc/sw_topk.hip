// sw_topk.hip — device top-K of a score vector, for the multi-GPU exchange
// (each rank's best K (score, id) go to one RCCL all-gather).
//
// Hits are ordered by score descending, then global id ascending; both fold
// into one int64 key (score << 32 | (2^31 - 1 - id)) sorted descending.
// Radix select: a workgroup holds a chunk of keys in registers (16 per
// thread: 4,096 keys for 256 threads, 16,384 for 1,024), finds its k-th largest key with 8-bit digit histograms in
// LDS — starting at the highest bit where the chunk's keys differ, stopping
// as soon as the keys left at the chosen digit are exactly the ones still
// needed — and writes the k keys at or above it (equal keys, i.e. padding,
// by ticket).  The stage repeats on the survivors (chunks x k keys) until one
// chunk remains, whose workgroup also sorts its k keys (bitonic in LDS).  No
// host synchronisation: every stage's size is known from n and k.
//
// Workgroup size: the ranking runs beside the next scan (bench.py's exchange
// stream), whose workgroups hold every CU with 2 waves per SIMD at 256 VGPRs
// each.  A 1,024-thread workgroup (4 waves per SIMD at 66 VGPRs, 72 with the
// allocation granule) fits nowhere until the scan's grid has drained: its
// kernel traces showed the ranking's first stage taking a whole scan (6.15 ms
// on C2).  For k <= 1,024 the stages run 256-thread workgroups (one wave per
// SIMD), which fit in the registers one finished scan workgroup leaves:
// C2 (570k scores, k = 100) ranks in 3 launches (140 chunks, 4, 1); larger k
// keeps 1,024 threads (a stage must keep fewer keys than it reads).
#include "sw_kernels.h"

namespace swk {

constexpr int kTopkPer = 16;      // keys per thread
constexpr int kTopkMaxK = 4096;
constexpr int kTopkSmallK = 1024;  // k up to this: 256-thread workgroups (4,096-key chunks)
constexpr int64_t kKeyPad = INT64_MIN;

__device__ __forceinline__ int64_t make_key(int32_t score, int64_t id) {
    return (static_cast<int64_t>(score) << 32) | ((int64_t{1} << 31) - 1 - id);
}
// order-preserving map of the signed keys onto uint64 (pad -> 0)
__device__ __forceinline__ uint64_t key_ord(int64_t k) { return static_cast<uint64_t>(k) ^ (uint64_t{1} << 63); }
__device__ __forceinline__ int64_t key_of(uint64_t u) { return static_cast<int64_t>(u ^ (uint64_t{1} << 63)); }

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const int lo = __shfl_xor(static_cast<int>(v & 0xffffffffu), m);
    const int hi = __shfl_xor(static_cast<int>(v >> 32), m);
    return (static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) | static_cast<uint32_t>(lo);
}

// in_scores != nullptr: keys are built from scores (ids = id_base + i, or
// ids[i] when an id map is given: a rank's residue-balanced shard of one
// database holds scattered global ids; BY_ID: entry i is scores[ids[i]], the
// score array of a scan, indexed by result id); otherwise they come from
// in_keys.  FINAL: one workgroup, sorted output.
template <int kTopkThreads, bool FINAL, bool BY_ID = false>
__global__ __launch_bounds__(kTopkThreads) void sw_topk_select(const int32_t* __restrict__ in_scores,
                                                              const int64_t* __restrict__ in_keys, int64_t n,
                                                              int64_t id_base, const int32_t* __restrict__ ids,
                                                              int k, int64_t* __restrict__ out) {
    __shared__ uint32_t hist[256];
    __shared__ uint64_t red[2][kTopkThreads / 64];
    __shared__ int ctl[5];  // digit, keys above it, keys at it, output slot, tie ticket
    __shared__ int64_t sorted[FINAL ? kTopkMaxK : 1];
    constexpr int kTopkChunk = kTopkThreads * kTopkPer;  // keys per workgroup
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int64_t start = static_cast<int64_t>(blockIdx.x) * kTopkChunk;
    const int m = static_cast<int>(min(static_cast<int64_t>(kTopkChunk), n - start));  // keys in this chunk
    uint64_t u[kTopkPer];
    uint64_t all_and = ~uint64_t{0}, all_or = 0;
#pragma unroll
    for (int j = 0; j < kTopkPer; ++j) {
        const int i = j * kTopkThreads + t;
        u[j] = 0;
        if (i < m) {
            const int64_t g = start + i;
            if (BY_ID) u[j] = key_ord(make_key(in_scores[ids[g]], ids[g]));
            else u[j] = key_ord(in_scores ? make_key(in_scores[g], ids ? ids[g] : id_base + g) : in_keys[g]);
            all_and &= u[j];
            all_or |= u[j];
        }
    }
    if (t == 0) {
        ctl[3] = 0;
        ctl[4] = 0;
    }
    auto emit = [&](uint64_t v) {
        const int pos = atomicAdd(&ctl[3], 1);
        if (FINAL) sorted[pos] = key_of(v);
        else out[static_cast<int64_t>(blockIdx.x) * k + pos] = key_of(v);
    };
    if (m <= k) {  // workgroup-uniform: every key survives
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kTopkPer; ++j)
            if (j * kTopkThreads + t < m) emit(u[j]);
    } else {
        // bits above the highest one where the chunk's keys differ are common
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            all_and &= shfl_xor64(all_and, off);
            all_or |= shfl_xor64(all_or, off);
        }
        if (lane == 0) {
            red[0][wave] = all_and;
            red[1][wave] = all_or;
        }
        __syncthreads();
        all_and = red[0][0];
        all_or = red[1][0];
        for (int w = 1; w < kTopkThreads / 64; ++w) {
            all_and &= red[0][w];
            all_or |= red[1][w];
        }
        const uint64_t diff = all_and ^ all_or;
        int remaining = k;  // keys still to take among those matching prefix
        uint64_t mask = ~uint64_t{0}, prefix = all_and;
        if (diff) {
            const int top = 63 - __clzll(static_cast<long long>(diff));
            mask = top == 63 ? 0 : ~((uint64_t{1} << (top + 1)) - 1);
            prefix = all_and & mask;
            for (int s = top - 7;; s -= 8) {
                const int sh = max(s, 0);
                const uint32_t dmask = (1u << (s >= 0 ? 8 : 8 + s)) - 1;
                if (t < 256) hist[t] = 0;
                __syncthreads();
#pragma unroll
                for (int j = 0; j < kTopkPer; ++j)
                    if (j * kTopkThreads + t < m && (u[j] & mask) == prefix)
                        atomicAdd(&hist[static_cast<uint32_t>(u[j] >> sh) & dmask], 1u);
                __syncthreads();
                if (wave == 0) {
                    // the digit d where the count of keys at digits >= d
                    // first reaches `remaining` (lane l holds bins 4l..4l+3)
                    const uint32_t h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2],
                                   h3 = hist[4 * lane + 3];
                    const int sum = static_cast<int>(h0 + h1 + h2 + h3);
                    int suf = sum;
#pragma unroll
                    for (int off = 1; off < 64; off <<= 1) {
                        const int v = __shfl_down(suf, off);
                        if (lane + off < 64) suf += v;
                    }
                    int run = suf - sum;  // keys at lanes above this one
                    const int hb[4] = {static_cast<int>(h0), static_cast<int>(h1), static_cast<int>(h2),
                                       static_cast<int>(h3)};
#pragma unroll
                    for (int b = 3; b >= 0; --b) {
                        if (run < remaining && run + hb[b] >= remaining) {
                            ctl[0] = 4 * lane + b;
                            ctl[1] = run;
                            ctl[2] = hb[b];
                        }
                        run += hb[b];
                    }
                }
                __syncthreads();
                const int d = ctl[0];
                remaining -= ctl[1];
                prefix |= static_cast<uint64_t>(d) << sh;
                mask |= static_cast<uint64_t>(dmask) << sh;
                if (ctl[2] == remaining || sh == 0) break;  // workgroup-uniform
                __syncthreads();  // ctl and hist are rewritten by the next pass
            }
        }
        // keys above the prefix all survive; of those at it, `remaining`
        // (all of them unless they are equal keys, i.e. padding)
#pragma unroll
        for (int j = 0; j < kTopkPer; ++j) {
            if (j * kTopkThreads + t >= m) continue;
            const uint64_t mu = u[j] & mask;
            if (mu > prefix) emit(u[j]);
            else if (mu == prefix && atomicAdd(&ctl[4], 1) < remaining) emit(u[j]);
        }
    }
    if constexpr (!FINAL) {
        __syncthreads();
        for (int i = min(m, k) + t; i < k; i += kTopkThreads) out[static_cast<int64_t>(blockIdx.x) * k + i] = kKeyPad;
    } else {
        int P = 1;
        while (P < k) P <<= 1;
        __syncthreads();
        for (int i = min(m, k) + t; i < P; i += kTopkThreads) sorted[i] = kKeyPad;
        __syncthreads();
        // bitonic sort of P keys, descending
        for (int size = 2; size <= P; size <<= 1) {
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                for (int i = t; i < P / 2; i += kTopkThreads) {
                    const int lo = 2 * i - (i & (stride - 1));
                    const int hi = lo + stride;
                    const bool desc = ((lo & size) == 0);
                    const int64_t a = sorted[lo], b = sorted[hi];
                    if ((a < b) == desc) {
                        sorted[lo] = b;
                        sorted[hi] = a;
                    }
                }
                __syncthreads();
            }
        }
        for (int i = t; i < k; i += kTopkThreads) out[i] = sorted[i];
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
static hipError_t launch_topk_t(const int32_t* scores, const int64_t* keys, int64_t n, int64_t id_base,
                                const int32_t* ids, int k, int64_t* out, int64_t* work, hipStream_t s, bool by_id) {
    constexpr int64_t chunk = T * kTopkPer;
    const int32_t* sc = scores;
    const int64_t* kin = keys;
    int64_t cur = n;
    int64_t* w = work;
    while (cur > chunk) {  // each stage keeps k of every chunk's keys (k <= chunk / 4)
        const int64_t chunks = (cur + chunk - 1) / chunk;
        if (sc && by_id)
            hipLaunchKernelGGL((sw_topk_select<T, false, true>), dim3(static_cast<unsigned>(chunks)), dim3(T), 0, s, sc,
                               kin, cur, id_base, ids, k, w);
        else
            hipLaunchKernelGGL((sw_topk_select<T, false>), dim3(static_cast<unsigned>(chunks)), dim3(T), 0, s, sc, kin,
                               cur, id_base, ids, k, w);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        sc = nullptr;
        kin = w;
        cur = chunks * k;
        w += cur;
    }
    if (sc && by_id)
        hipLaunchKernelGGL((sw_topk_select<T, true, true>), dim3(1), dim3(T), 0, s, sc, kin, cur, id_base, ids, k, out);
    else
        hipLaunchKernelGGL((sw_topk_select<T, true>), dim3(1), dim3(T), 0, s, sc, kin, cur, id_base,
                           sc ? ids : nullptr, k, out);
    return hipGetLastError();
}

hipError_t launch_topk(const int32_t* scores, const int64_t* keys, int64_t n, int64_t id_base, const int32_t* ids,
                       int k, int64_t* out, int64_t* work, hipStream_t s, bool by_id) {
    if (k <= 0 || k > kTopkMaxK || (by_id && (!scores || !ids))) return hipErrorInvalidValue;
    return k <= kTopkSmallK ? launch_topk_t<256>(scores, keys, n, id_base, ids, k, out, work, s, by_id)
                            : launch_topk_t<1024>(scores, keys, n, id_base, ids, k, out, work, s, by_id);
}

}  // namespace swk
