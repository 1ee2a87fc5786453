// Microbenchmark: wave64 VALU throughput of the instructions a SW cell can be
// built from (gfx950).  8 independent chains per lane, full occupancy.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHAINS 8
#define ITERS 4096

#define BODY(INSTR)                                                                    \
    __global__ __launch_bounds__(256) void k_##INSTR(uint32_t* out, uint32_t seed) {  \
        uint32_t v[CHAINS];                                                           \
        for (int c = 0; c < CHAINS; ++c) v[c] = seed + threadIdx.x * 7 + c;           \
        uint32_t y = seed ^ 0x1234567u, z = seed + 99u;                              \
        for (int it = 0; it < ITERS; ++it) {                                          \
            _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) INSTR_##INSTR(v[c]);   \
        }                                                                             \
        uint32_t acc = 0;                                                             \
        for (int c = 0; c < CHAINS; ++c) acc ^= v[c];                                 \
        out[blockIdx.x * 256 + threadIdx.x] = acc;                                    \
    }

#define INSTR_add_u32(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_max3_i32(x) asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z))
#define INSTR_sub_clamp(x) asm volatile("v_sub_u32 %0, %0, %1 clamp" : "+v"(x) : "v"(y))
#define INSTR_add_sdwa(x) asm volatile("v_add_u32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(x) : "v"(y))
#define INSTR_pk_add_u16(x) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_pk_max_i16(x) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_pk_sub_u16_clamp(x) asm volatile("v_pk_sub_u16 %0, %0, %1 clamp" : "+v"(x) : "v"(y))
#define INSTR_add_f32(x) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_max3_f32(x) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z))
#define INSTR_fma_f32(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z))
#define INSTR_max_i32(x) asm volatile("v_max_i32 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_bfi(x) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(x) : "v"(y), "v"(z))
#define INSTR_perm(x) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z))
#define INSTR_max_i16(x) asm volatile("v_max_i16 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_max_u16_sdwa(x) asm volatile("v_max_u16_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1" : "+v"(x) : "v"(y))

BODY(add_u32) BODY(max3_i32) BODY(sub_clamp) BODY(add_sdwa) BODY(pk_add_u16) BODY(pk_max_i16)
BODY(pk_sub_u16_clamp) BODY(add_f32) BODY(max3_f32) BODY(fma_f32) BODY(max_i32) BODY(bfi) BODY(perm)
BODY(max_i16) BODY(max_u16_sdwa)

#define INSTR_max_u32(x) asm volatile("v_max_u32 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_min_i32(x) asm volatile("v_min_i32 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_max_f32(x) asm volatile("v_max_f32 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_add_u16(x) asm volatile("v_add_u16 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_sub_u16_clamp(x) asm volatile("v_sub_u16_e64 %0, %0, %1 clamp" : "+v"(x) : "v"(y))
#define INSTR_max_u16(x) asm volatile("v_max_u16 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_max_i16_e64(x) asm volatile("v_max_i16_e64 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_cvt_ubyte1(x) asm volatile("v_cvt_f32_ubyte1 %0, %1" : "=v"(x) : "v"(x))
#define INSTR_add3_u32(x) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z))
#define INSTR_med3_i32(x) asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z))
#define INSTR_mov_b32(x) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(x))
#define INSTR_cndmask(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(y))
#define INSTR_lshrrev(x) asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(x))
#define INSTR_and_b32(x) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_bfe_i32(x) asm volatile("v_bfe_i32 %0, %0, 8, 8" : "+v"(x))
#define INSTR_add_i16(x) asm volatile("v_add_u16_e64 %0, %0, %1 clamp" : "+v"(x) : "v"(y))
#define INSTR_sub_i32_clamp(x) asm volatile("v_sub_i32 %0, %0, %1 clamp" : "+v"(x) : "v"(y))
#define INSTR_add_co_u32(x) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x) : "v"(y) : "vcc")
#define INSTR_max_i16_sdwa_w1(x) asm volatile("v_max_i16_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1" : "+v"(x) : "v"(y))
#define INSTR_max_f16(x) asm volatile("v_max_f16 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_pk_max_f16(x) asm volatile("v_pk_max_f16 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_add_lshl(x) asm volatile("v_add_lshl_u32 %0, %0, %1, 1" : "+v"(x) : "v"(y))
#define INSTR_dot2(x) asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(x) : "v"(y), "v"(z))
BODY(max_u32) BODY(min_i32) BODY(max_f32) BODY(add_u16) BODY(sub_u16_clamp) BODY(max_u16) BODY(max_i16_e64) BODY(cvt_ubyte1) BODY(add3_u32) BODY(med3_i32) BODY(mov_b32) BODY(cndmask) BODY(lshrrev) BODY(and_b32) BODY(bfe_i32) BODY(add_i16) BODY(sub_i32_clamp) BODY(add_co_u32) BODY(max_i16_sdwa_w1) BODY(max_f16) BODY(pk_max_f16) BODY(add_lshl) BODY(dot2)

#define INSTR_max3_i16(x) asm volatile("v_max3_i16 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z))
#define INSTR_max3_u16(x) asm volatile("v_max3_u16 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z))
#define INSTR_med3_i16(x) asm volatile("v_med3_i16 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z))
#define INSTR_add_u16_opsel_hi(x) asm volatile("v_mad_u16 %0, %1, 1, %0 op_sel:[1,0,0,0]" : "+v"(x) : "v"(y))
#define INSTR_max_i16_opsel_hi(x) asm volatile("v_add_i16 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_max3_i16_opsel(x) asm volatile("v_max3_i16 %0, %0, %1, %2 op_sel:[0,1,0,0]" : "+v"(x) : "v"(y), "v"(z))
#define INSTR_sub_u16_clamp_e64(x) asm volatile("v_sub_u16_e64 %0, %0, %1 clamp" : "+v"(x) : "v"(y))
#define INSTR_add_u16_e32(x) asm volatile("v_add_u16_e32 %0, %0, %1" : "+v"(x) : "v"(y))
#define INSTR_mad_u16(x) asm volatile("v_mad_u16 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z))
BODY(max3_i16) BODY(max3_u16) BODY(med3_i16) BODY(add_u16_opsel_hi) BODY(max_i16_opsel_hi) BODY(max3_i16_opsel) BODY(sub_u16_clamp_e64) BODY(add_u16_e32) BODY(mad_u16)


// per-"cell" instruction mixes (8 independent chains so latency is hidden)
#define INSTR_mix_cell_i32(x) asm volatile("v_add_u32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n v_max3_i32 %0, %0, %1, %2\n v_sub_u32 %0, %0, %1 clamp\n v_max3_i32 %2, %2, %0, %1" : "+v"(x), "+v"(z) : "v"(y))
#define INSTR_mix_cell_p32(x) asm volatile("v_add_u32 %0, %0, %1\n v_max3_i32 %0, %0, %1, %2\n v_sub_u32 %0, %0, %1 clamp\n v_max3_i32 %2, %2, %0, %1" : "+v"(x), "+v"(z) : "v"(y))
#define INSTR_mix_cell_16(x) asm volatile("v_add_u16 %0, %0, %1\n v_max_i16 %0, %0, %1\n v_max_i16 %0, %0, %2\n v_sub_u16_e64 %0, %0, %1 clamp\n v_max_i16 %2, %2, %0" : "+v"(x), "+v"(z) : "v"(y))
#define INSTR_mix_pk_dualq(x) asm volatile("v_pk_add_u16 %0, %0, %1\n v_pk_max_i16 %0, %0, %1\n v_pk_max_i16 %0, %0, %2\n v_pk_sub_u16 %0, %0, %1 clamp\n v_pk_max_i16 %2, %2, %0" : "+v"(x), "+v"(z) : "v"(y))
BODY(mix_cell_i32) BODY(mix_cell_p32) BODY(mix_cell_16) BODY(mix_pk_dualq)

// v_pk_fma_f32 / v_pk_add_f32 need 64-bit register pairs
__global__ __launch_bounds__(256) void k_pk_add_f32(uint32_t* out, uint32_t seed) {
    double v[CHAINS];
    for (int c = 0; c < CHAINS; ++c) v[c] = seed + threadIdx.x * 7 + c;
    double y = seed * 0.5;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(v[c]) : "v"(y));
    }
    double acc = 0;
    for (int c = 0; c < CHAINS; ++c) acc += v[c];
    out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)acc;
}


__global__ void probe(uint32_t* o) {
    uint32_t x = 0xABCD0005u, y = 0x12340003u, z = 0x7777FFFEu, r;
    asm volatile("v_add_u16_e64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y)); o[0] = r;
    asm volatile("v_mad_u16 %0, %1, 1, %2 op_sel:[1,0,0,0]" : "=v"(r) : "v"(y), "v"(x)); o[1] = r;
    asm volatile("v_max3_i16 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z)); o[2] = r;
    asm volatile("v_sub_u16_e64 %0, %1, %2 clamp" : "=v"(r) : "v"(y), "v"(x)); o[3] = r;
    asm volatile("v_max_i16 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y)); o[4] = r;
    uint32_t w = 0xFFFF0000u | 0x0002u; // low = 2
    asm volatile("v_sub_u16_e64 %0, %1, %2 clamp" : "=v"(r) : "v"(w), "v"(x)); o[5] = r; // 2 - 5 -> 0
    uint32_t neg = 0x0000FFFDu; // low16 = -3
    asm volatile("v_max3_i16 %0, %1, %2, %3" : "=v"(r) : "v"(neg), "v"(w), "v"(neg)); o[6] = r; // max(-3, 2, -3) = 2
    uint32_t hi = 0x00070000u;
    asm volatile("v_max3_i16 %0, %1, %2, %3 op_sel:[0,1,0,0]" : "=v"(r) : "v"(w), "v"(hi), "v"(neg)); o[7] = r; // max(2, 7, -3) = 7
}

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
    struct { const char* name; kfn f; } ks[] = {
        {"v_add_u32", k_add_u32}, {"v_sub_u32 clamp", k_sub_clamp}, {"v_max_i16", k_max_i16},
        {"sub_u16_clamp", k_sub_u16_clamp}, {"v_max3_i32", k_max3_i32}, {"v_pk_max_i16", k_pk_max_i16},
        {"mix_cell_i32", k_mix_cell_i32}, {"mix_cell_p32", k_mix_cell_p32}, {"mix_cell_16", k_mix_cell_16},
        {"mix_pk_dualq", k_mix_pk_dualq},
    };
    int dev = 0;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, dev);
    const int cus = p.multiProcessorCount;
    const int wpc = getenv("WAVES_PER_SIMD") ? atoi(getenv("WAVES_PER_SIMD")) : 8;
    const int blocks = cus * wpc;  // wpc x 256 threads per CU = wpc waves per SIMD
    uint32_t* out;
    hipMalloc(&out, blocks * 256 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    printf("CUs %d, clock %d kHz\n", cus, p.clockRate);
    {
        uint32_t h[8];
        hipLaunchKernelGGL(probe, dim3(1), dim3(1), 0, 0, out);
        hipMemcpy(h, out, 32, hipMemcpyDeviceToHost);
        const char* names[8] = {"add_u16 5+3", "add_u16 op_sel hi(0x1234)+5", "max3_i16(5,3,-2)", "sub_u16 clamp 3-5",
                                "max_i16(5,3)", "sub_u16 clamp 2-5", "max3_i16(-3,2,-3)", "max3_i16 opsel(2,hi7,-3)"};
        for (int i = 0; i < 8; ++i) printf("probe %-30s = 0x%08x\n", names[i], h[i]);
    }
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1u);
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1u);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double instr = 5.0 * blocks * 4 /*waves*/ * (double)ITERS * CHAINS;  // wave-instructions
        const double per_simd_per_s = instr / (cus * 4.0) / (ms * 1e-3);
        printf("%-28s %8.3f ms  wave-instr/SIMD/ns %.4f  => cycles/wave-instr @2.4GHz %.2f\n", k.name, ms,
               per_simd_per_s / 1e9, 2.4e9 / per_simd_per_s);
    }
    return 0;
}
