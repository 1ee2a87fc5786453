/*
 * SWSolver_char.h — drop-in for the reference's src/SWSolver_char.h.
 *
 * Identical declaration (reference SWSolver_char.h:7,9).  The reference body
 * (SWSolver_char.cu:193-280) does not compile; this build gives
 * it the scores of smith_waterman_cuda (golden-pinned) and returns them as a
 * new vector in file (id) order.
 */
#ifndef SWSOLVERCHAR_H
#define SWSOLVERCHAR_H

#include <vector>

#include "FASTAParsers.h"

typedef std::pair<int, int> seqid_score;

std::vector<seqid_score> smith_waterman_cuda_char(FASTAQuery &query, FASTADatabase &db);

#endif /* SWSOLVERCHAR_H */
