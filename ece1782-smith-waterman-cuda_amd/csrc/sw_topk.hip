// sw_topk.hip — device top-K of a score vector, for the multi-GPU exchange
// (each rank's best K (score, id) go to one RCCL all-gather).
//
// Hits are ordered by score descending, then global id ascending; both fold
// into one int64 key (score << 32 | (2^31 - 1 - id)) sorted descending.
// Each workgroup sorts a chunk of kChunk keys in LDS (bitonic) and keeps its
// best K; the stage repeats on the survivors until a single chunk remains.
// No host synchronisation: every stage's size is known from n and K.
#include "sw_kernels.h"

namespace swk {

constexpr int kTopkChunk = 8192;   // keys per workgroup (64 KiB of LDS)
constexpr int kTopkThreads = 512;
constexpr int64_t kKeyPad = INT64_MIN;

__device__ __forceinline__ int64_t make_key(int32_t score, int64_t id) {
    return (static_cast<int64_t>(score) << 32) | ((int64_t{1} << 31) - 1 - id);
}

// in_scores != nullptr: stage 0 builds keys from scores (ids = id_base + i);
// otherwise keys come from in_keys.
__global__ __launch_bounds__(kTopkThreads) void sw_topk_stage(const int32_t* __restrict__ in_scores,
                                                              const int64_t* __restrict__ in_keys, int64_t n,
                                                              int64_t id_base, int k, int64_t* __restrict__ out) {
    __shared__ int64_t key[kTopkChunk];
    const int64_t start = static_cast<int64_t>(blockIdx.x) * kTopkChunk;
    for (int i = threadIdx.x; i < kTopkChunk; i += kTopkThreads) {
        const int64_t g = start + i;
        int64_t v = kKeyPad;
        if (g < n) v = in_scores ? make_key(in_scores[g], id_base + g) : in_keys[g];
        key[i] = v;
    }
    __syncthreads();
    // bitonic sort, descending
    for (int size = 2; size <= kTopkChunk; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = threadIdx.x; i < kTopkChunk / 2; i += kTopkThreads) {
                const int lo = 2 * i - (i & (stride - 1));
                const int hi = lo + stride;
                const bool desc = ((lo & size) == 0);
                const int64_t a = key[lo], b = key[hi];
                if ((a < b) == desc) {
                    key[lo] = b;
                    key[hi] = a;
                }
            }
            __syncthreads();
        }
    }
    for (int i = threadIdx.x; i < k; i += kTopkThreads) out[static_cast<int64_t>(blockIdx.x) * k + i] = key[i];
}

// Workspace bytes sw_topk_device needs for n inputs and k outputs.
size_t topk_workspace_bytes(int64_t n, int k) {
    size_t total = 0;
    int64_t cur = n;
    while (cur > kTopkChunk) {
        const int64_t chunks = (cur + kTopkChunk - 1) / kTopkChunk;
        cur = chunks * k;
        total += static_cast<size_t>(cur) * sizeof(int64_t);
    }
    return total + 256;
}

hipError_t launch_topk(const int32_t* scores, const int64_t* keys, int64_t n, int64_t id_base, int k,
                       int64_t* out, int64_t* work, hipStream_t s) {
    if (k <= 0 || k > kTopkChunk / 2) return hipErrorInvalidValue;
    const int32_t* sc = scores;
    const int64_t* kin = keys;
    int64_t cur = n;
    int64_t* w = work;
    while (cur > kTopkChunk) {
        const int64_t chunks = (cur + kTopkChunk - 1) / kTopkChunk;
        hipLaunchKernelGGL(sw_topk_stage, dim3(static_cast<unsigned>(chunks)), dim3(kTopkThreads), 0, s, sc, kin,
                           cur, id_base, k, w);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        sc = nullptr;
        kin = w;
        cur = chunks * k;
        w += cur;
    }
    hipLaunchKernelGGL(sw_topk_stage, dim3(1), dim3(kTopkThreads), 0, s, sc, kin, cur, id_base, k, out);
    return hipGetLastError();
}

}  // namespace swk
