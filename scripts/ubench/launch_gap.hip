// launch_gap.hip — what a kernel launch, an event record and a cross-stream
// wait cost on the GPU's command processor between two dependent kernels
// (same stream).  Each variant enqueues N tiny kernels (grid G x 256) with
// the given packets between them and reports the GPU time per kernel.
//   build: hipcc --offload-arch=gfx950 -O2 -o launch_gap launch_gap.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

__global__ void tiny(int* p, int n) {
    if (blockIdx.x == 0 && threadIdx.x == 0) p[0] += n;
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? std::atoi(argv[1]) : 2000;
    int* d;
    CK(hipMalloc(&d, 64));
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    std::vector<hipEvent_t> et(N), en(N);
    for (int i = 0; i < N; ++i) {
        CK(hipEventCreate(&et[i]));
        CK(hipEventCreateWithFlags(&en[i], hipEventDisableTiming));
    }
    hipEvent_t done;
    CK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    CK(hipEventRecord(done, s2));
    CK(hipDeviceSynchronize());
    const char* names[] = {"kernels only (grid 1)", "kernels only (grid 512)", "kernels only (grid 3000)",
                           "+ timing event record", "+ 2 timing event records", "+ no-timing event record",
                           "+ wait on a completed event of another stream", "+ timing record + wait"};
    for (int v = 0; v < 8; ++v) {
        const int grid = v == 1 ? 512 : v == 2 ? 3000 : 1;
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipDeviceSynchronize());
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < N; ++i) {
                hipLaunchKernelGGL(tiny, dim3(grid), dim3(256), 0, s, d, i);
                if (v == 3 || v == 4 || v == 7) CK(hipEventRecord(et[i], s));
                if (v == 4) CK(hipEventRecord(en[i], s));
                if (v == 5) CK(hipEventRecord(en[i], s));
                if (v == 6 || v == 7) CK(hipStreamWaitEvent(s, done, 0));
            }
            const auto t1 = std::chrono::steady_clock::now();
            CK(hipStreamSynchronize(s));
            const auto t2 = std::chrono::steady_clock::now();
            if (rep == 1)
                std::printf("%-48s %7.2f us per kernel (host enqueue %.2f us)\n", names[v],
                            std::chrono::duration<double, std::micro>(t2 - t0).count() / N,
                            std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
        }
    }
    return 0;
}
