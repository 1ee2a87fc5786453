// sw_align.hip — GPU traceback of chosen hits.
//
// The reference prints alignments only from its CPU program: cpu.cpp:47-70
// fills H with a direction per cell (left, then up, then diagonal, each
// taken only on a STRICT improvement over the running value that starts at
// 0), keeps the first strict maximum in row-major order, and walks back
// while the cell is non-zero (cpu.cpp:76-108).  sw_align_linear reproduces
// those rules exactly for any substitution matrix and a linear gap, one hit
// per workgroup; sw_align_affine extends them to affine gaps (below):
//
//  * fill: an anti-diagonal sweep (cells i + j = d are independent); the
//    three most recent diagonals of H live in a per-hit global scratch
//    (3 x (qlen+1) int32, so query length is unbounded), the direction of
//    every cell is stored as one byte in a diagonal-major array T[d][i]
//    (consecutive threads write consecutive bytes);
//  * best cell: per-thread (value, i, j) maxima with the row-major tie rule,
//    reduced across the workgroup;
//  * walk back: one thread follows T from the best cell, writing the ops
//    (M aligned pair, I query residue vs gap, D subject residue vs gap).
//
// Cost is O(|q| |s|) per hit — meant for the top hits of a scan, not the
// database.
#include "sw_kernels.h"

namespace swk {

constexpr int kAlignThreads = 256;

struct Best {
    int h, i, j;
};

// (h, i, j) ordering of cpu.cpp's scan: larger h wins; on equal h the cell
// met first in row-major order (smaller i, then smaller j); h == 0 never
// replaces the initial (0, 0, 0).
__device__ __forceinline__ bool better(const Best& x, const Best& y) {
    if (x.h != y.h) return x.h > y.h;
    if (x.h == 0) return false;
    return x.i < y.i || (x.i == y.i && x.j < y.j);
}

// The walk back from the best cell (thread 0), both gap models: H's source
// in bits 0-1 of a direction byte, E / F extending in bits 2 / 3 (always 0
// under linear gaps, where every E / F opens).
__device__ void align_walk(const AlignArgs& a, const Best& bb, const uint8_t* T, int W1, int hit) {
    int i = bb.i, j = bb.j, state = 0;  // 0: H, 1: in an E run (left), 2: in an F run (up)
    int64_t n = 0;
    char* ops = a.ops ? a.ops + static_cast<int64_t>(hit) * a.ops_stride : nullptr;
    while (i > 0 && j > 0) {
        const int t = T[static_cast<int64_t>(i + j) * W1 + i];
        char op;
        if (state == 0) {
            const int src = t & 3;
            if (src == 0) break;  // a zero cell (H = 0 has no source)
            if (src != 3) {
                state = src;
                continue;
            }
            op = 'M';
            --i;
            --j;
        } else if (state == 1) {
            op = 'D';
            state = (t & 4) ? 1 : 0;
            --j;
        } else {
            op = 'I';
            state = (t & 8) ? 2 : 0;
            --i;
        }
        if (ops && n < a.ops_stride) ops[n] = op;
        ++n;
    }
    if (ops) {
        const int64_t m = n < a.ops_stride ? n : a.ops_stride;
        for (int64_t k = 0; k < m / 2; ++k) {
            const char c = ops[k];
            ops[k] = ops[m - 1 - k];
            ops[m - 1 - k] = c;
        }
    }
    int32_t* r = a.out + static_cast<int64_t>(hit) * 6;
    r[0] = bb.h;
    r[1] = i + 1;  // q_begin (1-based)
    r[2] = bb.i;   // q_end
    r[3] = j + 1;  // s_begin
    r[4] = bb.j;   // s_end
    r[5] = static_cast<int32_t>(n);
}

__global__ __launch_bounds__(kAlignThreads) void sw_align_linear(AlignArgs a) {
    __shared__ int8_t smat[640];
    __shared__ Best red[kAlignThreads];
    const int hit = blockIdx.x;
    const int tid = threadIdx.x;
    const int qlen = a.qlen;
    const int64_t soff = a.subj_off[hit];
    const int slen = static_cast<int>(a.subj_off[hit + 1] - soff);
    const uint8_t* __restrict__ q = a.query;
    const uint8_t* __restrict__ s = a.subj + soff;
    const int W1 = qlen + 1;
    int32_t* Hb = a.hbuf + static_cast<int64_t>(hit) * 3 * W1;
    uint8_t* T = a.dirs + a.dirs_off[hit];
    const int gap = a.gap;

    for (int k = tid; k < 625; k += kAlignThreads) smat[k] = a.mat[k];
    for (int k = tid; k < 3 * W1; k += kAlignThreads) Hb[k] = 0;
    __syncthreads();

    Best b = {0, 0, 0};
    for (int d = 2; d <= qlen + slen; ++d) {
        const int lo = max(1, d - slen);
        const int hi = min(qlen, d - 1);
        int32_t* cur = Hb + (d % 3) * W1;
        const int32_t* p1 = Hb + ((d + 2) % 3) * W1;  // diagonal d-1
        const int32_t* p2 = Hb + ((d + 1) % 3) * W1;  // diagonal d-2
        for (int i = lo + tid; i <= hi; i += kAlignThreads) {
            const int j = d - i;
            int h = 0, t = 0;
            const int left = p1[i] - gap;  // H(i, j-1)
            if (left > h) { h = left; t = 1; }
            const int up = p1[i - 1] - gap;  // H(i-1, j)
            if (up > h) { h = up; t = 2; }
            const int dg = p2[i - 1] + smat[25 * q[i - 1] + s[j - 1]];  // H(i-1, j-1) + S
            if (dg > h) { h = dg; t = 3; }
            cur[i] = h;
            T[static_cast<int64_t>(d) * W1 + i] = static_cast<uint8_t>(t);
            const Best c = {h, i, j};
            if (better(c, b)) b = c;
        }
        __syncthreads();  // diagonal d complete before d+1 reads it
    }

    red[tid] = b;
    __syncthreads();
    for (int w = kAlignThreads / 2; w > 0; w >>= 1) {
        if (tid < w && better(red[tid + w], red[tid])) red[tid] = red[tid + w];
        __syncthreads();
    }
    if (tid == 0) align_walk(a, red[0], T, W1, hit);
}

// Affine gaps (Gotoh; a k-gap costs gap + (k - 1) gap_extend).  The reference
// has no affine traceback, so the tie order is this build's own, cpu.cpp's
// carried over (oracle swo_align_affine states the same): E(i,j) opens from
// H(i,j-1) unless extending E(i,j-1) is STRICTLY better (F likewise down the
// column), H takes E, then F, then the diagonal on strict improvements over
// 0, the first strict maximum in row-major order ends the alignment.  The
// sweep keeps three diagonals of H and two of E and F (7 x (qlen + 1) int32
// per hit); E(i,j) reads diagonal d-1 at i, F(i,j) at i-1.
__global__ __launch_bounds__(kAlignThreads) void sw_align_affine(AlignArgs a) {
    __shared__ int8_t smat[640];
    __shared__ Best red[kAlignThreads];
    constexpr int NEG = -(1 << 29);
    const int hit = blockIdx.x;
    const int tid = threadIdx.x;
    const int qlen = a.qlen;
    const int64_t soff = a.subj_off[hit];
    const int slen = static_cast<int>(a.subj_off[hit + 1] - soff);
    const uint8_t* __restrict__ q = a.query;
    const uint8_t* __restrict__ s = a.subj + soff;
    const int W1 = qlen + 1;
    int32_t* Hb = a.hbuf + static_cast<int64_t>(hit) * 7 * W1;
    int32_t* Eb = Hb + 3 * W1;
    int32_t* Fb = Eb + 2 * W1;
    uint8_t* T = a.dirs + a.dirs_off[hit];
    const int go = a.gap, ge = a.gap_extend;

    for (int k = tid; k < 625; k += kAlignThreads) smat[k] = a.mat[k];
    for (int k = tid; k < 3 * W1; k += kAlignThreads) Hb[k] = 0;
    for (int k = tid; k < 4 * W1; k += kAlignThreads) Eb[k] = NEG;  // E and F
    __syncthreads();

    Best b = {0, 0, 0};
    for (int d = 2; d <= qlen + slen; ++d) {
        const int lo = max(1, d - slen);
        const int hi = min(qlen, d - 1);
        int32_t* cur = Hb + (d % 3) * W1;
        const int32_t* p1 = Hb + ((d + 2) % 3) * W1;  // H, diagonal d-1
        const int32_t* p2 = Hb + ((d + 1) % 3) * W1;  // H, diagonal d-2
        int32_t* ec = Eb + (d & 1) * W1;
        const int32_t* ep = Eb + ((d + 1) & 1) * W1;  // E, diagonal d-1
        int32_t* fc = Fb + (d & 1) * W1;
        const int32_t* fp = Fb + ((d + 1) & 1) * W1;  // F, diagonal d-1
        for (int i = lo + tid; i <= hi; i += kAlignThreads) {
            const int j = d - i;
            int t = 0;
            int e = p1[i] - go;                           // open from H(i, j-1)
            if (ep[i] - ge > e) { e = ep[i] - ge; t |= 4; }  // extend E(i, j-1)
            int f = p1[i - 1] - go;                       // open from H(i-1, j)
            if (fp[i - 1] - ge > f) { f = fp[i - 1] - ge; t |= 8; }
            int h = 0;
            if (e > h) { h = e; t = (t & 12) | 1; }
            if (f > h) { h = f; t = (t & 12) | 2; }
            const int dg = p2[i - 1] + smat[25 * q[i - 1] + s[j - 1]];
            if (dg > h) { h = dg; t = (t & 12) | 3; }
            cur[i] = h;
            ec[i] = e;
            fc[i] = f;
            T[static_cast<int64_t>(d) * W1 + i] = static_cast<uint8_t>(t);
            const Best c = {h, i, j};
            if (better(c, b)) b = c;
        }
        __syncthreads();  // diagonal d complete before d+1 reads it
    }

    red[tid] = b;
    __syncthreads();
    for (int w = kAlignThreads / 2; w > 0; w >>= 1) {
        if (tid < w && better(red[tid + w], red[tid])) red[tid] = red[tid + w];
        __syncthreads();
    }
    if (tid == 0) align_walk(a, red[0], T, W1, hit);
}

hipError_t launch_align(const AlignArgs& a, hipStream_t s) {
    if (a.n <= 0) return hipSuccess;
    if (a.gap_extend != a.gap)
        hipLaunchKernelGGL(sw_align_affine, dim3(a.n), dim3(kAlignThreads), 0, s, a);
    else
        hipLaunchKernelGGL(sw_align_linear, dim3(a.n), dim3(kAlignThreads), 0, s, a);
    return hipGetLastError();
}

}  // namespace swk
