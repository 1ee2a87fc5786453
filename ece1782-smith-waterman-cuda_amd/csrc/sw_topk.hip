// sw_topk.hip — device top-K of a score vector, for the multi-GPU exchange
// (each rank's best K (score, id) go to one RCCL all-gather).
//
// Hits are ordered by score descending, then global id ascending; both fold
// into one int64 key (score << 32 | (2^31 - 1 - id)) sorted descending.
// Each workgroup sorts a chunk of CH keys in LDS (bitonic) and keeps its
// best K; the stage repeats on the survivors until a single chunk remains.
// No host synchronisation: every stage's size is known from n and K.
// CH = 2048 (256 threads) when K <= 1024: ~n/2048 workgroups fill the chip
// and the network is 66 passes deep; 8192-key chunks (91 passes, 70
// workgroups for 570k scores) took 2 x 92 us per step on C2.
#include "sw_kernels.h"

namespace swk {

constexpr int kTopkChunk = 8192;   // largest chunk: keys per workgroup (64 KiB of LDS)
constexpr int64_t kKeyPad = INT64_MIN;

__device__ __forceinline__ int64_t make_key(int32_t score, int64_t id) {
    return (static_cast<int64_t>(score) << 32) | ((int64_t{1} << 31) - 1 - id);
}

// in_scores != nullptr: stage 0 builds keys from scores (ids = id_base + i);
// otherwise keys come from in_keys.
template <int CH, int NT>
__global__ __launch_bounds__(NT) void sw_topk_stage(const int32_t* __restrict__ in_scores,
                                                   const int64_t* __restrict__ in_keys, int64_t n, int64_t id_base,
                                                   int k, int64_t* __restrict__ out) {
    __shared__ int64_t key[CH];
    const int64_t start = static_cast<int64_t>(blockIdx.x) * CH;
    for (int i = threadIdx.x; i < CH; i += NT) {
        const int64_t g = start + i;
        int64_t v = kKeyPad;
        if (g < n) v = in_scores ? make_key(in_scores[g], id_base + g) : in_keys[g];
        key[i] = v;
    }
    __syncthreads();
    // bitonic sort, descending
    for (int size = 2; size <= CH; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = threadIdx.x; i < CH / 2; i += NT) {
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
    for (int i = threadIdx.x; i < k; i += NT) out[static_cast<int64_t>(blockIdx.x) * k + i] = key[i];
}

static int chunk_for(int k) { return k <= 1024 ? 2048 : kTopkChunk; }

// Workspace bytes sw_topk_device needs for n inputs and k outputs.
size_t topk_workspace_bytes(int64_t n, int k) {
    const int CH = chunk_for(k);
    size_t total = 0;
    int64_t cur = n;
    while (cur > CH) {
        const int64_t chunks = (cur + CH - 1) / CH;
        cur = chunks * k;
        total += static_cast<size_t>(cur) * sizeof(int64_t);
    }
    return total + 256;
}

hipError_t launch_topk(const int32_t* scores, const int64_t* keys, int64_t n, int64_t id_base, int k,
                       int64_t* out, int64_t* work, hipStream_t s) {
    if (k <= 0 || k > kTopkChunk / 2) return hipErrorInvalidValue;
    const int CH = chunk_for(k);
    auto stage = [&](unsigned grid, const int32_t* sc, const int64_t* kin, int64_t cnt, int64_t* dst) {
        if (CH == 2048)
            hipLaunchKernelGGL((sw_topk_stage<2048, 256>), dim3(grid), dim3(256), 0, s, sc, kin, cnt, id_base, k, dst);
        else
            hipLaunchKernelGGL((sw_topk_stage<kTopkChunk, 512>), dim3(grid), dim3(512), 0, s, sc, kin, cnt, id_base,
                               k, dst);
    };
    const int32_t* sc = scores;
    const int64_t* kin = keys;
    int64_t cur = n;
    int64_t* w = work;
    while (cur > CH) {
        const int64_t chunks = (cur + CH - 1) / CH;
        stage(static_cast<unsigned>(chunks), sc, kin, cur, w);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        sc = nullptr;
        kin = w;
        cur = chunks * k;
        w += cur;
    }
    stage(1, sc, kin, cur, out);
    return hipGetLastError();
}

}  // namespace swk
