/*
 * sw_oracle.c — CPU restatement of the reference Smith-Waterman scan.
 *
 * TEST INFRASTRUCTURE ONLY (see sw_oracle.h).  Plain C, scalar int32
 * arithmetic, no SIMD tricks: the point is to be obviously the textbook
 * recurrence the reference's golden files were produced with.
 *
 * Parity pins (tests/test_oracle.py):
 *   - golden scores test/reference/{P01008,P02232}.txt lines 0..110 against
 *     the 111 SwissProt records of data/dbs/uniprot_subset.dat;
 *   - the maximum cell of the matrix printed by src/cpu.cpp (built from the
 *     untouched reference source into oracle/_ref/cpu_ref by oracle/Makefile).
 */
#include "sw_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* ------------------------------------------------------------------ */
/* Alphabet: SWSolver.cu:17-41 (A=0 ... V=19, B=20, J=21, Z=22, X=23,  */
/* STAR=24) and convertStringToFloat, SWSolver.cu:91-120.              */
/* ------------------------------------------------------------------ */
static const char kLetters[] = "ARNDCQEGHILKMFPSTWYVBJZX";

int swo_encode_char(int ch) {
    for (int k = 0; k < 24; ++k)
        if (kLetters[k] == ch) return k;
    return SWO_STAR; /* SWSolver.cu:119 — anything else scores as '*' */
}

int64_t swo_encode(const char* in, int64_t n, uint8_t* out) {
    int8_t lut[256];
    for (int c = 0; c < 256; ++c) lut[c] = (int8_t)swo_encode_char(c);
    for (int64_t i = 0; i < n; ++i) out[i] = (uint8_t)lut[(unsigned char)in[i]];
    return n;
}

/* ------------------------------------------------------------------ */
/* Matrices (code order ARNDCQEGHILKMFPSTWYVBJZX*).                     */
/* ------------------------------------------------------------------ */
/* BLOSUM50 as tabulated in SWSolver.cu:54-81 (the '*' row and column are
 * all zero there, and X scores -1 against every letter). */
static const int8_t kBlosum50Ref[25 * 25] = {
/*      A   R   N   D   C   Q   E   G   H   I   L   K   M   F   P   S   T   W   Y   V   B   J   Z   X   * */
/*A*/   5, -2, -1, -2, -1, -1, -1,  0, -2, -1, -2, -1, -1, -3, -1,  1,  0, -3, -2,  0, -2, -2, -1, -1,  0,
/*R*/  -2,  7, -1, -2, -4,  1,  0, -3,  0, -4, -3,  3, -2, -3, -3, -1, -1, -3, -1, -3, -1, -3,  0, -1,  0,
/*N*/  -1, -1,  7,  2, -2,  0,  0,  0,  1, -3, -4,  0, -2, -4, -2,  1,  0, -4, -2, -3,  5, -4,  0, -1,  0,
/*D*/  -2, -2,  2,  8, -4,  0,  2, -1, -1, -4, -4, -1, -4, -5, -1,  0, -1, -5, -3, -4,  6, -4,  1, -1,  0,
/*C*/  -1, -4, -2, -4, 13, -3, -3, -3, -3, -2, -2, -3, -2, -2, -4, -1, -1, -5, -3, -1, -3, -2, -3, -1,  0,
/*Q*/  -1,  1,  0,  0, -3,  7,  2, -2,  1, -3, -2,  2,  0, -4, -1,  0, -1, -1, -1, -3,  0, -3,  4, -1,  0,
/*E*/  -1,  0,  0,  2, -3,  2,  6, -3,  0, -4, -3,  1, -2, -3, -1, -1, -1, -3, -2, -3,  1, -3,  5, -1,  0,
/*G*/   0, -3,  0, -1, -3, -2, -3,  8, -2, -4, -4, -2, -3, -4, -2,  0, -2, -3, -3, -4, -1, -4, -2, -1,  0,
/*H*/  -2,  0,  1, -1, -3,  1,  0, -2, 10, -4, -3,  0, -1, -1, -2, -1, -2, -3,  2, -4,  0, -3,  0, -1,  0,
/*I*/  -1, -4, -3, -4, -2, -3, -4, -4, -4,  5,  2, -3,  2,  0, -3, -3, -1, -3, -1,  4, -4,  4, -3, -1,  0,
/*L*/  -2, -3, -4, -4, -2, -2, -3, -4, -3,  2,  5, -3,  3,  1, -4, -3, -1, -2, -1,  1, -4,  4, -3, -1,  0,
/*K*/  -1,  3,  0, -1, -3,  2,  1, -2,  0, -3, -3,  6, -2, -4, -1,  0, -1, -3, -2, -3,  0, -3,  1, -1,  0,
/*M*/  -1, -2, -2, -4, -2,  0, -2, -3, -1,  2,  3, -2,  7,  0, -3, -2, -1, -1,  0,  1, -3,  2, -1, -1,  0,
/*F*/  -3, -3, -4, -5, -2, -4, -3, -4, -1,  0,  1, -4,  0,  8, -4, -3, -2,  1,  4, -1, -4,  1, -4, -1,  0,
/*P*/  -1, -3, -2, -1, -4, -1, -1, -2, -2, -3, -4, -1, -3, -4, 10, -1, -1, -4, -3, -3, -2, -3, -1, -1,  0,
/*S*/   1, -1,  1,  0, -1,  0, -1,  0, -1, -3, -3,  0, -2, -3, -1,  5,  2, -4, -2, -2,  0, -3,  0, -1,  0,
/*T*/   0, -1,  0, -1, -1, -1, -1, -2, -2, -1, -1, -1, -1, -2, -1,  2,  5, -3, -2,  0,  0, -1, -1, -1,  0,
/*W*/  -3, -3, -4, -5, -5, -1, -3, -3, -3, -3, -2, -3, -1,  1, -4, -4, -3, 15,  2, -3, -5, -2, -2, -1,  0,
/*Y*/  -2, -1, -2, -3, -3, -1, -2, -3,  2, -1, -1, -2,  0,  4, -3, -2, -2,  2,  8, -1, -3, -1, -2, -1,  0,
/*V*/   0, -3, -3, -4, -1, -3, -3, -4, -4,  4,  1, -3,  1, -1, -3, -2,  0, -3, -1,  5, -3,  2, -3, -1,  0,
/*B*/  -2, -1,  5,  6, -3,  0,  1, -1,  0, -4, -4,  0, -3, -4, -2,  0,  0, -5, -3, -3,  6, -4,  1, -1,  0,
/*J*/  -2, -3, -4, -4, -2, -3, -3, -4, -3,  4,  4, -3,  2,  1, -3, -3, -1, -2, -1,  2, -4,  4, -3, -1,  0,
/*Z*/  -1,  0,  0,  1, -3,  4,  5, -2,  0, -3, -3,  1, -1, -4, -1,  0, -1, -2, -2, -3,  1, -3,  5, -1,  0,
/*X*/  -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,  0,
/***/   0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,
};

/* NCBI BLOSUM62 (with J), same code order.  Not used by the reference; an
 * option of the build, and so "parity unpinned". */
static const int8_t kBlosum62[25 * 25] = {
/*      A   R   N   D   C   Q   E   G   H   I   L   K   M   F   P   S   T   W   Y   V   B   J   Z   X   * */
/*A*/   4, -1, -2, -2,  0, -1, -1,  0, -2, -1, -1, -1, -1, -2, -1,  1,  0, -3, -2,  0, -2, -1, -1,  0, -4,
/*R*/  -1,  5,  0, -2, -3,  1,  0, -2,  0, -3, -2,  2, -1, -3, -2, -1, -1, -3, -2, -3, -1, -2,  0, -1, -4,
/*N*/  -2,  0,  6,  1, -3,  0,  0,  0,  1, -3, -3,  0, -2, -3, -2,  1,  0, -4, -2, -3,  3, -3,  0, -1, -4,
/*D*/  -2, -2,  1,  6, -3,  0,  2, -1, -1, -3, -4, -1, -3, -3, -1,  0, -1, -4, -3, -3,  4, -3,  1, -1, -4,
/*C*/   0, -3, -3, -3,  9, -3, -4, -3, -3, -1, -1, -3, -1, -2, -3, -1, -1, -2, -2, -1, -3, -1, -3, -2, -4,
/*Q*/  -1,  1,  0,  0, -3,  5,  2, -2,  0, -3, -2,  1,  0, -3, -1,  0, -1, -2, -1, -2,  0, -2,  3, -1, -4,
/*E*/  -1,  0,  0,  2, -4,  2,  5, -2,  0, -3, -3,  1, -2, -3, -1,  0, -1, -3, -2, -2,  1, -3,  4, -1, -4,
/*G*/   0, -2,  0, -1, -3, -2, -2,  6, -2, -4, -4, -2, -3, -3, -2,  0, -2, -2, -3, -3, -1, -4, -2, -1, -4,
/*H*/  -2,  0,  1, -1, -3,  0,  0, -2,  8, -3, -3, -1, -2, -1, -2, -1, -2, -2,  2, -3,  0, -3,  0, -1, -4,
/*I*/  -1, -3, -3, -3, -1, -3, -3, -4, -3,  4,  2, -3,  1,  0, -3, -2, -1, -3, -1,  3, -3,  3, -3, -1, -4,
/*L*/  -1, -2, -3, -4, -1, -2, -3, -4, -3,  2,  4, -2,  2,  0, -3, -2, -1, -2, -1,  1, -4,  3, -3, -1, -4,
/*K*/  -1,  2,  0, -1, -3,  1,  1, -2, -1, -3, -2,  5, -1, -3, -1,  0, -1, -3, -2, -2,  0, -3,  1, -1, -4,
/*M*/  -1, -1, -2, -3, -1,  0, -2, -3, -2,  1,  2, -1,  5,  0, -2, -1, -1, -1, -1,  1, -3,  2, -1, -1, -4,
/*F*/  -2, -3, -3, -3, -2, -3, -3, -3, -1,  0,  0, -3,  0,  6, -4, -2, -2,  1,  3, -1, -3,  0, -3, -1, -4,
/*P*/  -1, -2, -2, -1, -3, -1, -1, -2, -2, -3, -3, -1, -2, -4,  7, -1, -1, -4, -3, -2, -2, -3, -1, -2, -4,
/*S*/   1, -1,  1,  0, -1,  0,  0,  0, -1, -2, -2,  0, -1, -2, -1,  4,  1, -3, -2, -2,  0, -2,  0,  0, -4,
/*T*/   0, -1,  0, -1, -1, -1, -1, -2, -2, -1, -1, -1, -1, -2, -1,  1,  5, -2, -2,  0, -1, -1, -1,  0, -4,
/*W*/  -3, -3, -4, -4, -2, -2, -3, -2, -2, -3, -2, -3, -1,  1, -4, -3, -2, 11,  2, -3, -4, -2, -3, -2, -4,
/*Y*/  -2, -2, -2, -3, -2, -1, -2, -3,  2, -1, -1, -2, -1,  3, -3, -2, -2,  2,  7, -1, -3, -1, -2, -1, -4,
/*V*/   0, -3, -3, -3, -1, -2, -2, -3, -3,  3,  1, -2,  1, -1, -2, -2,  0, -3, -1,  4, -3,  2, -2, -1, -4,
/*B*/  -2, -1,  3,  4, -3,  0,  1, -1,  0, -3, -4,  0, -3, -3, -2,  0, -1, -4, -3, -3,  4, -3,  1, -1, -4,
/*J*/  -1, -2, -3, -3, -1, -2, -3, -4, -3,  3,  3, -3,  2,  0, -3, -2, -1, -2, -1,  2, -3,  3, -3, -1, -4,
/*Z*/  -1,  0,  0,  1, -3,  3,  4, -2,  0, -3, -3,  1, -1, -3, -1,  0, -1, -3, -2, -2,  1, -3,  4, -1, -4,
/*X*/   0, -1, -1, -1, -2, -1, -1, -1, -1, -1, -1, -1, -1, -1, -2,  0,  0, -2, -1, -1, -1, -1, -1, -1, -4,
/***/  -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4,  1,
};

static int8_t kIdentity3[25 * 25];
static int kIdentityReady = 0;

const int8_t* swo_matrix(int id) {
    if (id == 0) return kBlosum50Ref;
    if (id == 1) return kBlosum62;
    if (id == 2) {
        if (!kIdentityReady) { /* cpu.cpp:6-8,22,57-59: equal +3, different -3 */
            for (int a = 0; a < 25; ++a)
                for (int b = 0; b < 25; ++b) kIdentity3[a * 25 + b] = (int8_t)(a == b ? 3 : -3);
            kIdentityReady = 1;
        }
        return kIdentity3;
    }
    return 0;
}

static inline int imax(int a, int b) { return a > b ? a : b; }

/* ------------------------------------------------------------------ */
/* Linear gap: SWSolver.cu:246 / cpu.cpp:43-74, one rolling row.        */
/* ------------------------------------------------------------------ */
int swo_score_linear(const uint8_t* q, int qlen, const uint8_t* s, int slen,
                     const int8_t* mat, int gap) {
    if (qlen <= 0 || slen <= 0) return 0;
    int* row = (int*)calloc((size_t)slen + 1, sizeof(int)); /* H(i-1, 0..slen) */
    int best = 0;
    for (int i = 1; i <= qlen; ++i) {
        const int8_t* mrow = mat + 25 * q[i - 1];
        int diag = 0;  /* H(i-1, j-1) */
        int left = 0;  /* H(i, j-1)   */
        for (int j = 1; j <= slen; ++j) {
            int up = row[j];
            int h = 0;
            h = imax(h, left - gap);
            h = imax(h, up - gap);
            h = imax(h, diag + mrow[s[j - 1]]);
            best = imax(best, h);
            diag = up;
            row[j] = h;
            left = h;
        }
    }
    free(row);
    return best;
}

/* ------------------------------------------------------------------ */
/* Affine gap (Gotoh).  With go == ge this equals the linear case.      */
/* ------------------------------------------------------------------ */
int swo_score_affine(const uint8_t* q, int qlen, const uint8_t* s, int slen,
                     const int8_t* mat, int go, int ge) {
    if (qlen <= 0 || slen <= 0) return 0;
    const int NEG = -(1 << 29);
    int* hrow = (int*)calloc((size_t)slen + 1, sizeof(int));
    int* frow = (int*)malloc(((size_t)slen + 1) * sizeof(int));
    for (int j = 0; j <= slen; ++j) frow[j] = NEG;
    int best = 0;
    for (int i = 1; i <= qlen; ++i) {
        const int8_t* mrow = mat + 25 * q[i - 1];
        int diag = 0, left = 0, e = NEG;
        for (int j = 1; j <= slen; ++j) {
            int up = hrow[j];
            e = imax(e - ge, left - go);
            int f = imax(frow[j] - ge, up - go);
            int h = imax(0, diag + mrow[s[j - 1]]);
            h = imax(h, imax(e, f));
            best = imax(best, h);
            diag = up;
            hrow[j] = h;
            frow[j] = f;
            left = h;
        }
    }
    free(hrow);
    free(frow);
    return best;
}

/* ------------------------------------------------------------------ */
/* cpu.cpp on raw bytes (cpu.cpp:18-74).                                 */
/* ------------------------------------------------------------------ */
int swo_score_raw_identity(const char* a, int alen, const char* b, int blen,
                           int match, int mismatch, int gap) {
    if (alen <= 0 || blen <= 0) return 0;
    int* row = (int*)calloc((size_t)blen + 1, sizeof(int));
    int best = 0;
    for (int i = 1; i <= alen; ++i) {
        int diag = 0, left = 0;
        for (int j = 1; j <= blen; ++j) {
            int up = row[j];
            int h = 0;
            h = imax(h, left - gap);
            h = imax(h, up - gap);
            h = imax(h, diag + (a[i - 1] == b[j - 1] ? match : mismatch));
            best = imax(best, h);
            diag = up;
            row[j] = h;
            left = h;
        }
    }
    free(row);
    return best;
}

/* ------------------------------------------------------------------ */
/* Traceback, cpu.cpp:43-103 tie rules.                                  */
/* ------------------------------------------------------------------ */
int swo_align_linear(const uint8_t* q, int qlen, const uint8_t* s, int slen,
                     const int8_t* mat, int gap, int* q_end, int* s_end,
                     int* q_begin, int* s_begin, char* ops, int ops_cap,
                     int* ops_len) {
    *q_end = *s_end = *q_begin = *s_begin = 0;
    *ops_len = 0;
    if (qlen <= 0 || slen <= 0) return 0;
    size_t W = (size_t)slen + 1;
    int* H = (int*)calloc(((size_t)qlen + 1) * W, sizeof(int));
    unsigned char* T = (unsigned char*)calloc(((size_t)qlen + 1) * W, 1);
    int best = 0, bi = 0, bj = 0;
    for (int i = 1; i <= qlen; ++i) {
        for (int j = 1; j <= slen; ++j) {
            int h = 0;
            unsigned char t = 0;
            if (H[i * W + j - 1] - gap > h) { h = H[i * W + j - 1] - gap; t = 1; }          /* left */
            if (H[(i - 1) * W + j] - gap > h) { h = H[(i - 1) * W + j] - gap; t = 2; }      /* up   */
            int d = H[(i - 1) * W + j - 1] + mat[25 * q[i - 1] + s[j - 1]];
            if (d > h) { h = d; t = 3; }                                                  /* diag */
            if (h > best) { best = h; bi = i; bj = j; }
            H[i * W + j] = h;
            T[i * W + j] = t;
        }
    }
    /* Walk back while the cell value is non-zero (cpu.cpp:80-103).  Ops are
     * written end->start then reversed: 'M' aligned pair, 'I' query residue
     * against a gap (move up), 'D' subject residue against a gap (move left). */
    int i = bi, j = bj, n = 0;
    while (i > 0 && j > 0 && H[i * W + j] != 0) {
        unsigned char t = T[i * W + j];
        char op;
        if (t == 1) { op = 'D'; --j; }
        else if (t == 2) { op = 'I'; --i; }
        else if (t == 3) { op = 'M'; --i; --j; }
        else break;
        if (n < ops_cap) ops[n] = op;
        ++n;
    }
    int m = n < ops_cap ? n : ops_cap;
    for (int k = 0; k < m / 2; ++k) { char c = ops[k]; ops[k] = ops[m - 1 - k]; ops[m - 1 - k] = c; }
    *ops_len = n;
    *q_end = bi; *s_end = bj;
    *q_begin = i + 1; *s_begin = j + 1;
    free(H);
    free(T);
    return best;
}

/* Affine traceback (Gotoh).  The reference has no affine path, so its tie
 * order is this build's own, cpu.cpp's carried over: E(i,j) = H(i,j-1) - go
 * unless extending, E(i,j-1) - ge, is STRICTLY better (the same for F down
 * the column); H takes, in order, E (left), F (up), the diagonal, each only
 * on a strict improvement over the running value that starts at 0; the end
 * cell is the first strict maximum in row-major order; the walk back from H
 * follows E / F runs to their opening cell and stops at a zero cell.  With
 * go == ge every E / F is an opening and this is swo_align_linear exactly.
 * Direction byte: bits 0-1 H's source (0 none, 1 E, 2 F, 3 diagonal), bit 2
 * E extends, bit 3 F extends.  Parity unpinned against the reference (it
 * prints no affine alignment): pinned to swo_score_affine and to the score
 * of its own path. */
int swo_align_affine(const uint8_t* q, int qlen, const uint8_t* s, int slen,
                     const int8_t* mat, int go, int ge, int* q_end, int* s_end,
                     int* q_begin, int* s_begin, char* ops, int ops_cap,
                     int* ops_len) {
    *q_end = *s_end = *q_begin = *s_begin = 0;
    *ops_len = 0;
    if (qlen <= 0 || slen <= 0) return 0;
    const int NEG = -(1 << 29);
    size_t W = (size_t)slen + 1;
    size_t cells = ((size_t)qlen + 1) * W;
    int* H = (int*)calloc(cells, sizeof(int));
    int* E = (int*)malloc(cells * sizeof(int));
    int* F = (int*)malloc(cells * sizeof(int));
    unsigned char* T = (unsigned char*)calloc(cells, 1);
    for (size_t k = 0; k < cells; ++k) E[k] = F[k] = NEG;
    int best = 0, bi = 0, bj = 0;
    for (int i = 1; i <= qlen; ++i) {
        for (int j = 1; j <= slen; ++j) {
            unsigned char t = 0;
            int e = H[i * W + j - 1] - go;
            if (E[i * W + j - 1] - ge > e) { e = E[i * W + j - 1] - ge; t |= 4; }
            int f = H[(i - 1) * W + j] - go;
            if (F[(i - 1) * W + j] - ge > f) { f = F[(i - 1) * W + j] - ge; t |= 8; }
            int h = 0;
            if (e > h) { h = e; t = (unsigned char)((t & 12) | 1); }
            if (f > h) { h = f; t = (unsigned char)((t & 12) | 2); }
            int d = H[(i - 1) * W + j - 1] + mat[25 * q[i - 1] + s[j - 1]];
            if (d > h) { h = d; t = (unsigned char)((t & 12) | 3); }
            if (h > best) { best = h; bi = i; bj = j; }
            H[i * W + j] = h;
            E[i * W + j] = e;
            F[i * W + j] = f;
            T[i * W + j] = t;
        }
    }
    int i = bi, j = bj, n = 0, state = 0; /* 0: H, 1: in an E run, 2: in an F run */
    while (i > 0 && j > 0) {
        unsigned char t = T[i * W + j];
        char op;
        if (state == 0) {
            int src = t & 3;
            if (src == 0 || H[i * W + j] == 0) break;
            if (src == 3) { op = 'M'; --i; --j; }
            else { state = src; continue; }
        } else if (state == 1) {
            op = 'D';
            state = (t & 4) ? 1 : 0;
            --j;
        } else {
            op = 'I';
            state = (t & 8) ? 2 : 0;
            --i;
        }
        if (n < ops_cap) ops[n] = op;
        ++n;
    }
    int m = n < ops_cap ? n : ops_cap;
    for (int k = 0; k < m / 2; ++k) { char c = ops[k]; ops[k] = ops[m - 1 - k]; ops[m - 1 - k] = c; }
    *ops_len = n;
    *q_end = bi; *s_end = bj;
    *q_begin = i + 1; *s_begin = j + 1;
    free(H); free(E); free(F); free(T);
    return best;
}

/* ------------------------------------------------------------------ */
/* Threaded whole-database scan (the CPU baseline).                      */
/* ------------------------------------------------------------------ */
typedef struct {
    const uint8_t* q; int qlen;
    const uint8_t* res; const int64_t* offs;
    int64_t n; const int8_t* mat; int go, ge;
    int32_t* out;
    volatile int64_t* next;  /* shared work counter */
} scan_job;

static void* scan_worker(void* arg) {
    scan_job* jb = (scan_job*)arg;
    const int64_t chunk = 64;
    for (;;) {
        int64_t k0 = __sync_fetch_and_add(jb->next, chunk);
        if (k0 >= jb->n) break;
        int64_t k1 = k0 + chunk < jb->n ? k0 + chunk : jb->n;
        for (int64_t k = k0; k < k1; ++k) {
            const uint8_t* s = jb->res + jb->offs[k];
            int slen = (int)(jb->offs[k + 1] - jb->offs[k]);
            jb->out[k] = (jb->go == jb->ge)
                ? swo_score_linear(jb->q, jb->qlen, s, slen, jb->mat, jb->go)
                : swo_score_affine(jb->q, jb->qlen, s, slen, jb->mat, jb->go, jb->ge);
        }
    }
    return 0;
}

void swo_scan(const uint8_t* q, int qlen, const uint8_t* res, const int64_t* offs,
              int64_t n, const int8_t* mat, int go, int ge, int32_t* out,
              int nthreads) {
    if (nthreads <= 0) nthreads = (int)sysconf(_SC_NPROCESSORS_ONLN);
    if (nthreads < 1) nthreads = 1;
    volatile int64_t next = 0;
    scan_job jb = {q, qlen, res, offs, n, mat, go, ge, out, &next};
    if (nthreads == 1) { scan_worker(&jb); return; }
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], 0, scan_worker, &jb);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], 0);
    free(th);
}
