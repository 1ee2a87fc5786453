// sw_synth.hip — synthetic databases generated in HBM (SURVEY.md §8d, config
// C4: "shards are generated on device from (seed, global id) with a
// counter-based RNG whose CPU restatement can regenerate any sampled id").
//
// Integer-only, so the host and any CPU restatement reproduce it bit for bit
// (synth.py counter_* functions, tests/test_synth_counter.py):
//   h(seed, id, k) = mix(seed * G1 + mix(id * G2 + k))         (splitmix64 mix)
//   length(id)     = LEN_TABLE[h(seed, id, LEN_SALT) >> 52]      (4096 log-normal quantiles)
//   residue(id, j) = RES_LUT[(h(seed, id, j >> 2) >> (16 * (j & 3))) & 0xffff]
// RES_LUT maps a uniform u16 to a residue code with Swiss-Prot frequencies.
// The host computes the lengths and the block layout (O(n)); these kernels
// write the residue bytes straight into the packed layouts, so a 6.25M-
// subject shard (2.25 GB) appears in HBM without a host copy or a PCIe
// transfer.
#include "sw_kernels.h"

namespace swk {

__host__ __device__ inline uint64_t syn_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__host__ __device__ inline uint64_t syn_hash(uint64_t seed, uint64_t id, uint64_t k) {
    return syn_mix(seed * 0x9E3779B97F4A7C15ull + syn_mix(id * 0xD6E8FEB86659FD93ull + k));
}

// inter part: one workgroup (64 lanes) per block, 16 residues per lane per
// group, one 16-byte store per lane per group
__global__ __launch_bounds__(64) void sw_synth_fill_inter(uint8_t* __restrict__ res, const uint64_t* __restrict__ blk_off,
                                                          const uint32_t* __restrict__ blk_groups,
                                                          const int32_t* __restrict__ lane_gid_lo,
                                                          const int32_t* __restrict__ lane_len, uint64_t seed,
                                                          int64_t id_base, const uint8_t* __restrict__ lut) {
    const int b = blockIdx.x;
    const int l = threadIdx.x;
    const int32_t local = lane_gid_lo[static_cast<int64_t>(b) * kLanes + l];
    const int32_t L = local >= 0 ? lane_len[static_cast<int64_t>(b) * kLanes + l] : 0;
    const uint64_t gid = static_cast<uint64_t>(id_base + local);
    const uint32_t G = blk_groups[b];
    uint8_t* base = res + blk_off[b] + static_cast<uint64_t>(l) * kGroupCols;
    for (uint32_t g = 0; g < G; ++g) {
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int j0 = static_cast<int>(g) * 16 + 4 * q;
            uint32_t word = 0;
            if (j0 < L) {
                const uint64_t h = syn_hash(seed, gid, static_cast<uint64_t>(j0 >> 2));
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t c = (j0 + e < L) ? lut[(h >> (16 * e)) & 0xffffu] : kPadCode;
                    word |= c << (8 * e);
                }
            } else {
                word = 0x19191919u;  // kPadCode
            }
            w[q] = word;
        }
        *reinterpret_cast<int4*>(base + static_cast<uint64_t>(g) * kGroupBytes) =
            make_int4(static_cast<int>(w[0]), static_cast<int>(w[1]), static_cast<int>(w[2]), static_cast<int>(w[3]));
    }
}

// intra part: plain per-subject layout (64-byte aligned starts, pad beyond)
__global__ __launch_bounds__(256) void sw_synth_fill_intra(uint8_t* __restrict__ lres, const uint64_t* __restrict__ loff,
                                                           const int32_t* __restrict__ llen,
                                                           const int32_t* __restrict__ lid, int32_t nlong,
                                                           uint64_t seed, int64_t id_base,
                                                           const uint8_t* __restrict__ lut) {
    const int k = blockIdx.x;
    if (k >= nlong) return;
    const int32_t L = llen[k];
    const uint64_t gid = static_cast<uint64_t>(id_base + lid[k]);
    uint8_t* dst = lres + loff[k];
    const int words = (L + 63) / 64 * 16;  // 4-residue words up to the 64-byte-aligned end
    for (int w = threadIdx.x; w < words; w += blockDim.x) {
        const int j0 = 4 * w;
        uint32_t word = 0;
        const uint64_t h = syn_hash(seed, gid, static_cast<uint64_t>(w));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint32_t c = (j0 + e < L) ? lut[(h >> (16 * e)) & 0xffffu] : kPadCode;
            word |= c << (8 * e);
        }
        *reinterpret_cast<uint32_t*>(dst + j0) = word;
    }
}

hipError_t launch_synth_fill(const SynthFill& f, hipStream_t s) {
    if (f.nblocks > 0) {
        hipLaunchKernelGGL(sw_synth_fill_inter, dim3(static_cast<unsigned>(f.nblocks)), dim3(kLanes), 0, s, f.res,
                           f.blk_off, f.blk_groups, f.lane_local, f.lane_len, f.seed, f.id_base, f.lut);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (f.nlong > 0) {
        hipLaunchKernelGGL(sw_synth_fill_intra, dim3(static_cast<unsigned>(f.nlong)), dim3(256), 0, s, f.lres, f.loff,
                           f.llen, f.lid, f.nlong, f.seed, f.id_base, f.lut);
        return hipGetLastError();
    }
    return hipSuccess;
}

uint64_t synth_hash(uint64_t seed, uint64_t id, uint64_t k) { return syn_hash(seed, id, k); }

}  // namespace swk
