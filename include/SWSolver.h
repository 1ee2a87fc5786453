/*
 * SWSolver.h — drop-in for the reference's src/SWSolver.h.
 *
 * Identical declarations (reference SWSolver.h:7,9).  The implementation
 * (ece1782-smith-waterman-cuda_amd/csrc/swsolver.cpp) scores on the MI355X
 * through the C ABI of include/sw_amd.h.  Semantics kept from
 * SWSolver.cu:266-404: the query is '/'-padded to a multiple of 8; (id, score)
 * pairs are APPENDED to `result` in descending padded-length order, file order
 * within a length.  Changed on purpose: exact int32 scores (the reference's
 * int16 storage overflows), no 1024-residue query cap (F6), and
 * a HIP failure throws std::runtime_error instead of going unnoticed.
 */
#ifndef SWSOLVER_H
#define SWSOLVER_H

#include <vector>

#include "FASTAParsers.h"

typedef std::pair<int, int> seqid_score;

void smith_waterman_cuda(FASTAQuery &query, FASTADatabase &db, std::vector<seqid_score> &result);

#endif /* SWSOLVER_H */
