// sw_rank.h — device-side ranking: the radix select and the bitonic sort of
// the top-K kernels (sw_topk.hip) as workgroup functions.
//
// Hits are ordered by score descending, then global id ascending; both fold
// into one int64 key (score << 32 | (2^31 - 1 - id)) sorted descending.  A
// workgroup holds up to T x PER keys in registers and finds their k-th
// largest with 8-bit digit histograms in LDS — starting at the highest bit
// where the keys differ, stopping as soon as the keys left at the chosen
// digit are exactly the ones still needed — then emits the k keys at or above
// it (equal keys, i.e. padding, by ticket).
#pragma once

#include "sw_kernels.h"

namespace swk {

constexpr int kTopkMaxK = 4096;
constexpr int64_t kKeyPad = INT64_MIN;

#if defined(__HIPCC__)
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

// Key g of a ranking input (TopkSrc, sw_kernels.h).
__device__ __forceinline__ uint64_t topk_key(const TopkSrc& s, int64_t g) {
    if (s.keys) return key_ord(s.keys[g]);
    const int64_t r = s.rid ? s.rid[g] : g;
    return key_ord(make_key(s.scores[r], s.gid ? s.gid[r] : s.id_base + r));
}

template <int T>
struct TopkLds {
    uint32_t hist[256];
    uint64_t red[2][T / 64];
    int ctl[5];  // digit, keys above it, keys at it, output slot, tie ticket
};

// The k largest of the m keys u[j] (index j T + t < m valid) of a T-thread
// workgroup: emit(pos, key) for each, pos = 0 .. min(m, k) - 1 in no order.
// Every thread calls it (barriers inside); L is the workgroup's LDS.
template <int T, int PER, class Emit>
__device__ __forceinline__ void topk_select(const uint64_t (&u)[PER], int m, int k, TopkLds<T>& L, Emit emit) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (t == 0) {
        L.ctl[3] = 0;
        L.ctl[4] = 0;
    }
    uint64_t all_and = ~uint64_t{0}, all_or = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j)
        if (j * T + t < m) {
            all_and &= u[j];
            all_or |= u[j];
        }
    if (m <= k) {  // workgroup-uniform: every key survives
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER; ++j)
            if (j * T + t < m) emit(atomicAdd(&L.ctl[3], 1), u[j]);
        __syncthreads();
        return;
    }
    // bits above the highest one where the keys differ are common
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        all_and &= shfl_xor64(all_and, off);
        all_or |= shfl_xor64(all_or, off);
    }
    if (lane == 0) {
        L.red[0][wave] = all_and;
        L.red[1][wave] = all_or;
    }
    __syncthreads();
    all_and = L.red[0][0];
    all_or = L.red[1][0];
    for (int w = 1; w < T / 64; ++w) {
        all_and &= L.red[0][w];
        all_or |= L.red[1][w];
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
            if (t < 256) L.hist[t] = 0;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < PER; ++j)
                if (j * T + t < m && (u[j] & mask) == prefix)
                    atomicAdd(&L.hist[static_cast<uint32_t>(u[j] >> sh) & dmask], 1u);
            __syncthreads();
            if (wave == 0) {
                // the digit d where the count of keys at digits >= d first
                // reaches `remaining` (lane l holds bins 4l..4l+3)
                const uint32_t h0 = L.hist[4 * lane], h1 = L.hist[4 * lane + 1], h2 = L.hist[4 * lane + 2],
                               h3 = L.hist[4 * lane + 3];
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
                        L.ctl[0] = 4 * lane + b;
                        L.ctl[1] = run;
                        L.ctl[2] = hb[b];
                    }
                    run += hb[b];
                }
            }
            __syncthreads();
            const int d = L.ctl[0];
            remaining -= L.ctl[1];
            prefix |= static_cast<uint64_t>(d) << sh;
            mask |= static_cast<uint64_t>(dmask) << sh;
            if (L.ctl[2] == remaining || sh == 0) break;  // workgroup-uniform
            __syncthreads();  // ctl and hist are rewritten by the next pass
        }
    }
    // keys above the prefix all survive; of those at it, `remaining` (all of
    // them unless they are equal keys, i.e. padding)
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        if (j * T + t >= m) continue;
        const uint64_t mu = u[j] & mask;
        if (mu > prefix) emit(atomicAdd(&L.ctl[3], 1), u[j]);
        else if (mu == prefix && atomicAdd(&L.ctl[4], 1) < remaining) emit(atomicAdd(&L.ctl[3], 1), u[j]);
    }
    __syncthreads();
}

// Bitonic sort (descending) of sorted[0 .. P), P = the power of two >= k,
// entries [n, P) padded first; then out[0 .. k) = the k best.
template <int T>
__device__ __forceinline__ void topk_sort_out(int64_t* sorted, int n, int k, int64_t* __restrict__ out) {
    const int t = threadIdx.x;
    int P = 1;
    while (P < k) P <<= 1;
    for (int i = n + t; i < P; i += T) sorted[i] = kKeyPad;
    __syncthreads();
    for (int size = 2; size <= P; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = t; i < P / 2; i += T) {
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
    for (int i = t; i < k; i += T) out[i] = sorted[i];
}

#endif

}  // namespace swk
