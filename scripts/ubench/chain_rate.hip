// Microbenchmark: the real DP dependency structure (one row chain per column,
// R rows in registers), compiler-generated code, int32 cell vs packed-16 cell
// (2 cells per instruction).  Reports cycles (@2.4 GHz) per CELL per SIMD.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef short s2 __attribute__((ext_vector_type(2)));
typedef unsigned short u2 __attribute__((ext_vector_type(2)));
#define R 32
#define COLS 2048

__device__ __forceinline__ int sx8(uint32_t w, int b) { return (int)(int8_t)(w >> (8 * b)); }

__global__ __launch_bounds__(256) void k_i32(const uint32_t* __restrict__ prof, int* out, uint32_t g) {
    int H[R];
    for (int r = 0; r < R; ++r) H[r] = 0;
    int best = 0;
    const int lane = threadIdx.x & 63;
    for (int j = 0; j < COLS; ++j) {
        uint32_t pw[R / 4];
#pragma unroll
        for (int q = 0; q < R / 4; ++q) pw[q] = __builtin_nontemporal_load(&prof[((j & 15) * (R / 4) + q) * 64 + lane]);
        int up = 0, diag = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int sc = sx8(pw[r >> 2], r & 3);
            const int h = (int)__builtin_elementwise_sub_sat((uint32_t)max(max(H[r], up), diag + sc), g);
            diag = H[r]; H[r] = h; up = h; best = max(best, h);
        }
        asm volatile("" : "+v"(best));
    }
    out[blockIdx.x * 256 + threadIdx.x] = best + H[5];
}

__global__ __launch_bounds__(256) void k_pk(const uint32_t* __restrict__ prof, int* out, uint32_t g2) {
    s2 H[R];
    for (int r = 0; r < R; ++r) H[r] = 0;
    s2 best = 0;
    const u2 g = __builtin_bit_cast(u2, g2);
    const int lane = threadIdx.x & 63;
    for (int j = 0; j < COLS / 2; ++j) {   // half the columns: 2 cells per op
        uint32_t pw[R];
#pragma unroll
        for (int q = 0; q < R; ++q) pw[q] = __builtin_nontemporal_load(&prof[((j & 15) * R + q) * 64 + lane]);
        s2 up = 0, diag = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const s2 a = diag + __builtin_bit_cast(s2, pw[r]);
            const s2 m = __builtin_elementwise_max(__builtin_elementwise_max(H[r], up), a);
            const s2 h = __builtin_bit_cast(s2, __builtin_elementwise_sub_sat(__builtin_bit_cast(u2, m), g));
            diag = H[r]; H[r] = h; up = h; best = __builtin_elementwise_max(best, h);
        }
        asm volatile("" : "+v"(best));
    }
    out[blockIdx.x * 256 + threadIdx.x] = __builtin_bit_cast(int, best) + __builtin_bit_cast(int, H[5]);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    uint32_t* prof;
    int* out;
    hipMalloc(&prof, 16 * R * 64 * 4 * 2);
    hipMemset(prof, 1, 16 * R * 64 * 4 * 2);
    hipMalloc(&out, cus * 8 * 256 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int wps : {1, 2, 3, 4, 6, 8}) {
        const int blocks = cus * wps;
        for (int kind = 0; kind < 2; ++kind) {
            auto launch = [&]() {
                if (kind == 0) hipLaunchKernelGGL(k_i32, dim3(blocks), dim3(256), 0, 0, prof, out, 2u);
                else hipLaunchKernelGGL(k_pk, dim3(blocks), dim3(256), 0, 0, prof, out, 0x00020002u);
            };
            launch();
            hipDeviceSynchronize();
            hipEventRecord(a);
            for (int r = 0; r < 3; ++r) launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double cells_per_simd = 3.0 * wps * 64.0 * COLS * R;  // per SIMD (wps waves each)
            printf("waves/SIMD %d %-4s %8.3f ms  cycles@2.4GHz per cell per SIMD %.2f\n", wps, kind ? "pk" : "i32",
                   ms, ms * 1e-3 * 2.4e9 / (cells_per_simd / 64.0));
        }
    }
    return 0;
}
