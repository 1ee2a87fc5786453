// Microbenchmark: gfx950 packed-fp16 ops for a Smith-Waterman cell
// (v_pk_maximum3_f16 is new in CDNA4) against the packed-int16 cell.
// 8 independent chains per lane; WAVES_PER_SIMD waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHAINS 8
#define ITERS 4096

#define BODY(INSTR)                                                                    \
    __global__ __launch_bounds__(256) void k_##INSTR(uint32_t* out, uint32_t seed) {  \
        uint32_t v[CHAINS], w[CHAINS];                                                \
        for (int c = 0; c < CHAINS; ++c) {                                            \
            v[c] = 0x3c003c00u + c;                                                   \
            w[c] = 0x40004000u + c;                                                   \
        }                                                                             \
        uint32_t y = 0x3c003c00u ^ (seed & 1), z = 0x00000000u;                       \
        for (int it = 0; it < ITERS; ++it) {                                          \
            _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) INSTR_##INSTR(v[c], w[c]); \
        }                                                                             \
        uint32_t acc = 0;                                                             \
        for (int c = 0; c < CHAINS; ++c) acc ^= v[c] ^ w[c];                          \
        out[blockIdx.x * 256 + threadIdx.x] = acc;                                    \
    }

#define INSTR_pk_maximum3_f16(x, u) asm volatile("v_pk_maximum3_f16 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z))
#define INSTR_pk_add_f16(x, u) asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_pk_max_f16(x, u) asm volatile("v_pk_max_f16 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_pk_max_i16(x, u) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(x) : "v"(y))
// one packed affine cell pair as the int16 kernel issues it (9 ops)
#define INSTR_cell_i16(x, u) asm volatile(                                              \
    "v_pk_add_u16 %0, %0, %2\n v_pk_max_i16 %1, %1, %0\n v_pk_max_i16 %0, %1, %2\n"   \
    "v_pk_sub_u16 %1, %0, %2 clamp\n v_pk_sub_u16 %0, %0, %2 clamp\n"                 \
    "v_pk_max_i16 %0, %0, %1\n v_pk_sub_u16 %1, %1, %2 clamp\n v_pk_max_i16 %1, %1, %0\n" \
    "v_pk_max_i16 %0, %0, %1" : "+v"(x), "+v"(u) : "v"(y))
// the same cell pair in fp16 with 3-input maxima (7.5 ops: best every 2nd row)
#define INSTR_cell_f16(x, u) asm volatile(                                              \
    "v_pk_add_f16 %0, %0, %2\n v_pk_maximum3_f16 %1, %1, %0, %2\n"                     \
    "v_pk_add_f16 %0, %1, %2\n v_pk_add_f16 %1, %1, %2\n v_pk_maximum3_f16 %1, %1, %0, %3\n" \
    "v_pk_add_f16 %0, %0, %2\n v_pk_maximum3_f16 %0, %0, %1, %3\n"                      \
    "v_pk_maximum3_f16 %1, %1, %0, %2" : "+v"(x), "+v"(u) : "v"(y), "v"(z))
BODY(pk_maximum3_f16) BODY(pk_add_f16) BODY(pk_max_f16) BODY(pk_max_i16) BODY(cell_i16) BODY(cell_f16)

__global__ void probe(uint32_t* o) {
    // fp16: 3.0 = 0x4200, 5.0 = 0x4500, -2.0 = 0xc000, 0 = 0x0000, 2047 = 0x67ff, 2048 = 0x6800
    uint32_t r;
    asm volatile("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(0x42004500u), "v"(0xc0000000u), "v"(0u));
    o[0] = r;  // expect lo max(5,0,0)=5 (0x4500), hi max(3,-2,0)=3 (0x4200)
    asm volatile("v_pk_add_f16 %0, %1, %2" : "=v"(r) : "v"(0x67ff4200u), "v"(0x3c00c000u));
    o[1] = r;  // lo 3 + -2 = 1 (0x3c00), hi 2047 + 1 = 2048 (0x6800)
    asm volatile("v_pk_add_f16 %0, %1, %2" : "=v"(r) : "v"(0x0000c000u), "v"(0x00004000u));
    o[2] = r;  // lo -2 + 2 = +0 (0x0000), hi 0 + 0 = 0
}

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
    struct { const char* name; kfn f; double ops; } ks[] = {
        {"v_pk_maximum3_f16", k_pk_maximum3_f16, 1}, {"v_pk_add_f16", k_pk_add_f16, 1},
        {"v_pk_max_f16", k_pk_max_f16, 1}, {"v_pk_max_i16", k_pk_max_i16, 1},
        {"cell pair int16 (9 ops)", k_cell_i16, 9}, {"cell pair fp16 (8 ops)", k_cell_f16, 8},
    };
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int wps = getenv("WAVES_PER_SIMD") ? atoi(getenv("WAVES_PER_SIMD")) : 8;
    const int blocks = cus * wps;
    uint32_t* out;
    hipMalloc(&out, blocks * 256 * 4);
    uint32_t h[3];
    hipLaunchKernelGGL(probe, dim3(1), dim3(1), 0, 0, out);
    hipMemcpy(h, out, 12, hipMemcpyDeviceToHost);
    printf("probe maximum3 %08x (expect 42004500)  add %08x (expect 68003c00)  add %08x (expect 00000000)\n", h[0],
           h[1], h[2]);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    printf("waves/SIMD %d\n", wps);
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1u);
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1u);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double groups = 5.0 * blocks * 4 * (double)ITERS * CHAINS;  // wave-level instruction groups
        const double per_simd = groups / (cus * 4.0) / (ms * 1e-3);
        printf("%-26s %8.3f ms  cycles per group @2.4GHz %.2f  (per op %.2f)\n", k.name, ms, 2.4e9 / per_simd,
               2.4e9 / per_simd / k.ops);
    }
    return 0;
}
