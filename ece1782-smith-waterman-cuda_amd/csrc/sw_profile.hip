// sw_profile.hip — the query profiles built on the device, from the query
// codes and the scoring matrix carried in the kernel arguments.
//
// The reference builds nothing per query: its kernel reads the BLOSUM50 table
// and the query from __constant__ memory (SWSolver.cu:54-81, 296-299, 246),
// one lookup per cell.  Here every scan kernel reads a per-query profile
// (prof[stored code][row] = S[q_row][code], + the gap for the linear kernels;
// the database stores code c as kStored[c], sw_kernels.h), so a
// scan starts by building it.  Built on the host and copied, each scan paid
// an H2D copy on the DMA engine plus the compute queue's wait for it, ~30-40
// us between two scans (rocprofv3 trace of C2's 1/8 share, profiles/r03_trace/);
// a kernel on the scan's own queue costs a few microseconds and needs no copy:
// the query and the matrix travel inside the launch's kernel arguments.
#include "sw_kernels.h"

namespace swk {

// One thread per (code, row) entry of rows [row0, row1).
__global__ __launch_bounds__(256) void sw_build_profile(ProfileArgs a) {
    if (blockIdx.x == 0 && threadIdx.x < 10) {  // the rescue lists' counters and heads, the merged
                                                // launch's work counter (first launch only)
        int32_t* p = a.reset[threadIdx.x];
        if (p) *p = threadIdx.x == 2 ? -1 : 0;
    }
    const int n = a.row1 - a.row0;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= kProfileRows * n) return;
    const int c = tid / n;  // the profile row: a STORED code (sw_kernels.h kStored)
    const int i = a.row0 + tid % n;
    const int v =
        (c >= kAlphabet || i >= a.qlen) ? a.bias : a.mat[kAlphabet * a.q[i - a.row0] + kCodeOf[c]] + a.bias;
    if (i < a.stride) {
        const size_t k = static_cast<size_t>(c) * a.stride + i;
        a.p8[k] = static_cast<int8_t>(v);
        if (a.p16) a.p16[k] = static_cast<int16_t>(v);
    }
    if (a.pin && i < a.qpad_intra) {
        // lane-slotted image of the int32 intra kernel: [chunk][code][lane][RIP]
        const int ch = i / (kLanes * a.ri), w = i % (kLanes * a.ri);
        const int t = w / a.ri, r = w % a.ri;
        int8_t* d = a.pin + ((static_cast<size_t>(ch) * kProfileRows + c) * kLanes + t) * a.rip;
        d[r] = static_cast<int8_t>(v);
        if (r == a.ri - 1)
            for (int p = a.ri; p < a.rip; ++p) d[p] = 0;
    }
}

hipError_t launch_build_profile(const ProfileArgs& a, hipStream_t s) {
    const int n = a.row1 - a.row0;
    if (n <= 0 || n > kProfQueryChunk) return hipErrorInvalidValue;
    const int threads = kProfileRows * n;
    hipLaunchKernelGGL(sw_build_profile, dim3((threads + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace swk
