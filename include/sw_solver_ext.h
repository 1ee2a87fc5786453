/*
 * sw_solver_ext.h — additions of this build to the C++ drop-in (SWSolver.h
 * itself stays identical to the reference's src/SWSolver.h:7,9).  Used by
 * lib/main and lib/sw_tests; the reference has no counterpart.
 */
#ifndef SW_SOLVER_EXT_H
#define SW_SOLVER_EXT_H

#include <stdint.h>

#include <string>
#include <vector>

#include "FASTAParsers.h"
#include "SWSolver.h"
#include "sw_amd.h"

/* Wall time of the last smith_waterman_cuda[_char] call, split as
 * flatten (map walk + encode on the host's cores), upload (pack + H2D into
 * resident shards) and scan (kernels + D2H of the scores). */
struct sw_solver_timing {
    double flatten_s;
    double upload_s;  /* sw_db_create: host packing + H2D of the database */
    double scan_s;
    int gpus;
    double init_s;    /* device start-up (HIP runtime, handle / group): the first call only */
};
sw_solver_timing sw_solver_last_timing();

/* Devices smith_waterman_cuda shards the database over (default: $SW_GPUS,
 * else 1; `main --gpus N`).  1 = the single-handle path. */
void sw_solver_set_gpus(int n);
/* The process-wide group behind the N > 1 path (created on first use), or
 * NULL when the solver runs on one GPU. */
sw_group* sw_solver_group();

/* main --make-db: the flattened database (reference order, record ids as
 * result ids, subjects as written: no '/' padding) written as a sw_db_save
 * file. */
void sw_save_fasta_db(FASTADatabase& fdb, const std::string& path);

/* Scoring of smith_waterman_cuda / smith_waterman_cuda_topk (the reference
 * hard-wires BLOSUM50, SWSolver.cu:54-81, and GAP_PENALTY 2, SWSolver.cu:7,
 * with "define affine penalty ?" left open at :8).  matrix625: 25x25 int8 in
 * code order (sw_amd.h), NULL = the reference's BLOSUM50; a gap of k
 * residues costs gap_open + (k - 1) gap_extend (open == extend: linear).
 * Throws std::invalid_argument outside 1..1000 / -100..100.  Until it is
 * called (or after sw_solver_reset_scoring) the solver scores exactly as the
 * reference, query padding included; a set scoring scans the query and
 * the subjects as written (without the '/' padding of SWSolver.cu:267-269
 * and FASTAParsers.h, which scores 0 only under the reference's table). */
void sw_solver_set_scoring(const int8_t* matrix625, int gap_open, int gap_extend);
void sw_solver_reset_scoring();
/* `spec` = "blosum50" (the reference's table), "blosum62", or a text file:
 * either 25 rows of 25 integers in code order ARNDCQEGHILKMFPSTWYVBJZX*, or
 * the NCBI layout (a header row of residue letters, then one row per letter,
 * '#' comments); letters an NCBI file leaves out (J in NCBI's BLOSUM62) score
 * as its X row / column.  False (and *err) on a bad file. */
bool sw_solver_read_matrix(const std::string& spec, int8_t out[625], std::string* err);

/* The k best subjects of the database for this query, score descending then
 * record id ascending, as (record id, score) pairs — the scan plus a device
 * top-K (sw_scan_topk; with several GPUs sw_group_topk: per-device top-K and
 * one RCCL all-gather), so only k results leave the GPU.  Fewer than k when
 * the database is smaller.  k > 4096 ranks every score on the host. */
std::vector<seqid_score> smith_waterman_cuda_topk(FASTAQuery& query, FASTADatabase& db, int k);

#endif /* SW_SOLVER_EXT_H */
