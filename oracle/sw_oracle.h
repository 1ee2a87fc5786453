/*
 * sw_oracle.h — CPU restatement of the reference Smith-Waterman scoring.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing on the product path (the HIP library,
 * the C++ drop-in, the CLI) links or calls this.  Only tests/, the smoke()
 * hook in __graft_entry__.py and bench.py's cpu_baseline leg may use it, and
 * only as the checker / the timed CPU baseline.
 *
 * Parity pin: the restatement reproduces test/reference/{P01008,P02232}.txt
 * (the reference's golden score files) exactly on the first 111 SwissProt
 * records, which ship as data/dbs/uniprot_subset.dat (fixtures under
 * tests/golden/, made by tests/golden/make_golden.py), and reproduces the
 * maximum of the matrix printed by the reference's own src/cpu.cpp (compiled
 * from the untouched reference source into oracle/_ref/ by oracle/Makefile)
 * on the pair fixtures in tests/golden/cpu_pairs.json.
 */
#ifndef SW_ORACLE_H
#define SW_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Residue alphabet of SWSolver.cu:17-41: A R N D C Q E G H I L K M F P S T W Y V
 * B J Z X *  -> codes 0..24.  Every other byte (U, O, lowercase, '/', '\r')
 * becomes '*' (code 24), as convertStringToFloat does (SWSolver.cu:91-120). */
#define SWO_ALPHABET 25
#define SWO_STAR 24

int swo_encode_char(int ch);
/* Encode n bytes; returns n. */
int64_t swo_encode(const char* in, int64_t n, uint8_t* out);

/* Built-in substitution matrices, 25x25 int8 row-major in code order.
 *   0: BLOSUM50 exactly as tabulated in SWSolver.cu:54-81 ('*' row/col = 0)
 *   1: BLOSUM62 (NCBI), '*' row/col = -4, '*'/'*' = 1 (option; unpinned)
 *   2: identity +3 / -3 (the cpu.cpp:6-8 scheme, applied to codes) */
const int8_t* swo_matrix(int id);

/* Score-only local alignment, linear gap: the recurrence of
 * SWSolver.cu:246 and cpu.cpp:43-74
 *   H(i,j) = max(0, H(i-1,j-1)+S[q_i][s_j], H(i,j-1)-gap, H(i-1,j)-gap)
 * returning max over all cells. i runs over the query (outer), j over the
 * subject (inner), as cpu.cpp:45-46. */
int swo_score_linear(const uint8_t* q, int qlen, const uint8_t* s, int slen,
                     const int8_t* mat, int gap);

/* Score-only local alignment, affine gap (Gotoh):
 *   E(i,j) = max(E(i,j-1)-ge, H(i,j-1)-go)
 *   F(i,j) = max(F(i-1,j)-ge, H(i-1,j)-go)
 *   H(i,j) = max(0, H(i-1,j-1)+S, E(i,j), F(i,j))
 * A gap of length k costs go + (k-1)*ge; go == ge == g is the linear case. */
int swo_score_affine(const uint8_t* q, int qlen, const uint8_t* s, int slen,
                     const int8_t* mat, int go, int ge);

/* The cpu.cpp program itself (cpu.cpp:16-74) on raw bytes: +match when bytes
 * are equal, +mismatch otherwise, linear gap.  Returns the maximum cell (the
 * value the traceback starts from, cpu.cpp:66-70,80-82). */
int swo_score_raw_identity(const char* a, int alen, const char* b, int blen,
                           int match, int mismatch, int gap);

/* Whole-database scan: score query q against n subjects whose encoded
 * residues are res[offs[k] .. offs[k+1]).  go == ge uses the linear
 * recurrence.  out[k] = score of subject k.  nthreads <= 0: all cores. */
void swo_scan(const uint8_t* q, int qlen, const uint8_t* res, const int64_t* offs,
              int64_t n, const int8_t* mat, int go, int ge, int32_t* out,
              int nthreads);

/* Optimal local alignment with traceback under the tie order of cpu.cpp:47-64
 * (strict '>' in order left, up, diagonal; first strict maximum cell,
 * cpu.cpp:66-70).  Linear gap only.  Writes the 1-based end cell and the
 * start cell (first aligned residue, 1-based) and the alignment length. */
int swo_align_linear(const uint8_t* q, int qlen, const uint8_t* s, int slen,
                     const int8_t* mat, int gap, int* q_end, int* s_end,
                     int* q_begin, int* s_begin, char* ops, int ops_cap,
                     int* ops_len);

/* The same under affine gaps (Gotoh, a k-gap costs go + (k-1) ge), with the
 * tie order described at its definition (this build's own: the reference
 * has no affine traceback).  go == ge gives swo_align_linear's result.   */
int swo_align_affine(const uint8_t* q, int qlen, const uint8_t* s, int slen,
                     const int8_t* mat, int go, int ge, int* q_end, int* s_end,
                     int* q_begin, int* s_begin, char* ops, int ops_cap,
                     int* ops_len);

#ifdef __cplusplus
}
#endif
#endif
