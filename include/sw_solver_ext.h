/*
 * sw_solver_ext.h — additions of this build to the C++ drop-in (SWSolver.h
 * itself stays identical to the reference's src/SWSolver.h:7,9).  Used by
 * lib/main and lib/sw_tests; the reference has no counterpart.
 */
#ifndef SW_SOLVER_EXT_H
#define SW_SOLVER_EXT_H

#include <string>

#include "FASTAParsers.h"
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
 * result ids) written as a sw_db_save file. */
void sw_save_fasta_db(FASTADatabase& fdb, const std::string& path);

#endif /* SW_SOLVER_EXT_H */
