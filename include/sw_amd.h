/*
 * sw_amd.h — C ABI of the MI355X Smith-Waterman database-scan library
 * (libswamd.so).  Plain pointers and sizes only; no C++ or torch types.
 *
 * This is the boundary the reference's scan path crosses.  The reference has
 * no FFI of its own: its one entry point is the C++ function
 *
 *     void smith_waterman_cuda(FASTAQuery&, FASTADatabase&,
 *                              std::vector<seqid_score>&);     SWSolver.h:9
 *
 * implemented at SWSolver.cu:266-404, plus the (uncompilable) char variant
 * SWSolver_char.h:9 / SWSolver_char.cu:193-280.  Those C++ signatures are
 * kept unchanged in include/SWSolver.h and include/SWSolver_char.h; they are
 * thin shims over the calls below.  Each call names the part of the
 * reference it replaces.
 *
 * Conventions
 *   - Residues are ENCODED bytes: codes 0..24 for A R N D C Q E G H I L K M F
 *     P S T W Y V B J Z X * (SWSolver.cu:17-41); every other input byte is
 *     '*' = 24 (convertStringToFloat, SWSolver.cu:91-120).  sw_encode()
 *     performs that mapping.
 *   - Scores are int32 (the reference's int16 storage overflows for the
 *     self-hits of the longest shipped queries).
 *   - Every call returns SW_OK (0) or a negative SW_E* code; a HIP failure
 *     is returned as SW_E_HIP and its text is kept for sw_last_error().
 *     Nothing fails silently (the reference checks no CUDA error,
 *     SWSolver.cu:276).
 *   - A handle is bound to one device and owns one HIP stream; calls on one
 *     handle are not re-entrant (neither is the reference: it keeps its
 *     query in __constant__ memory, SWSolver.cu:85-89).
 */
#ifndef SW_AMD_H
#define SW_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* libswamd.so is built with -fvisibility=hidden; only these are exported. */
#if defined(SW_AMD_BUILD)
#define SW_API __attribute__((visibility("default")))
#else
#define SW_API
#endif

#define SW_OK 0
#define SW_E_INVALID -1   /* bad argument */
#define SW_E_HIP -2       /* HIP runtime error (see sw_last_error) */
#define SW_E_NOMEM -3     /* host allocation failed */
#define SW_E_NODEVICE -4  /* no HIP device / kernel image for this GPU */
#define SW_E_UNSUPPORTED -5 /* valid request this build does not implement */
#define SW_E_IO -6          /* file could not be read / written / validated */
#define SW_E_DEVICE -7      /* a kernel reported an internal fault: the scores of the
                               handle's scans since the last successful call are not
                               trusted (see sw_last_error).  The device writes a
                               host-mapped word; the asynchronous entry points
                               (sw_scan_device, sw_scan_rank_device, the batch and
                               group forms) return before their kernels end, so a
                               fault is reported by the first call on the handle
                               after the faulting kernel has completed (the
                               synchronous sw_scan / sw_scan_topk / sw_scan_batch
                               report their own) */

#define SW_ALPHABET 25    /* residue codes 0..24 */
#define SW_CODE_STAR 24

/* Built-in substitution matrices (25x25 int8, code order). */
#define SW_MATRIX_BLOSUM50_REF 0  /* SWSolver.cu:54-81 exactly ('*' = 0) */
#define SW_MATRIX_BLOSUM62 1      /* NCBI BLOSUM62 (option, not in the reference) */
#define SW_MATRIX_IDENTITY3 2     /* +3/-3, the cpu.cpp:6-8 scheme */
#define SW_MATRIX_BLOSUM50_CHAR 3 /* the _char path's table (SWSolver_char.cu:22-49) as
                                     its lookup (:106-179) reads it: BLOSUM50_REF with
                                     '*' = -5 and '*'/'*' = 1 (its L->W typo at :35 is
                                     never read: the lookup orders the pair by range) */

typedef struct sw_scoring {
    const int8_t* matrix;  /* 625 int8 (row = query code, col = subject code);
                              NULL = SW_MATRIX_BLOSUM50_REF */
    int32_t gap_open;      /* cost of the first residue of a gap (> 0) */
    int32_t gap_extend;    /* cost of each further residue (> 0); equal to
                              gap_open = the reference's linear gap
                              (GAP_PENALTY 2, SWSolver.cu:7) */
} sw_scoring;

typedef struct sw_db_stats {
    int64_t n_subjects;      /* records in the database */
    int64_t residues;        /* sum of unpadded subject lengths */
    int64_t packed_cells;    /* residue columns actually scanned (64 lanes x
                                padded block widths) */
    int64_t n_blocks;        /* 64-subject blocks scanned by the inter-sequence kernel */
    int64_t n_long;          /* subjects routed to the intra-sequence kernel */
    int64_t device_bytes;    /* HBM held by the packed database */
    int32_t max_length;      /* longest subject */
    int32_t long_threshold;  /* subjects longer than this use the intra kernel */
    int32_t coop_blocks;     /* widest blocks the cooperative kernel took in the
                                most recent scan of this database (the split
                                depends on the scoring) */
    int64_t coop_residues;   /* unpadded residues in those blocks */
    int32_t max_id;          /* largest result id (-1 if empty): score arrays hold max_id+1 */
    int32_t pair_blocks;     /* widest blocks run by wave pairs (sw_inter_x2p) in
                                the most recent scan; in the default merged
                                launch they belong to the main inter kernel */
    int32_t pair_merged;     /* 1: pairs and single-wave blocks were one launch */
    int64_t pair_residues;   /* unpadded residues in the pair blocks */
} sw_db_stats;

typedef struct sw_timing {
    float inter_ms;     /* inter-sequence kernel(s), HIP events on the handle's stream */
    float intra_ms;     /* intra-sequence kernel(s) */
    float total_ms;     /* first launch to last completion of the last scan */
    int32_t rescued;    /* subjects re-scored at int32 after an int16 saturation */
    int32_t launches;   /* kernel launches in the last scan */
    float coop_ms;      /* cooperative wide-block kernel alone (events on its stream) */
    float wave_ms;      /* per-wave inter kernel alone (events on the handle's stream) */
} sw_timing;
/* A scan run as ONE merged longest-first launch (sw_last_kernel ends in
 * "+lpt": inter blocks and the long subjects' fp16 pass in one grid) reports
 * that launch as inter_ms and wave_ms and 0 as intra_ms.
 * In a batch (sw_scan_batch*), a query's rescue tail (re-scoring of flagged
 * subjects) may run on a tail stream beside the next query's scan: its time
 * is then outside that query's spans and inside a later query's total_ms;
 * the batch's sum covers all of it. */

typedef struct sw_handle sw_handle;
typedef struct sw_db sw_db;

/* ---- housekeeping ---------------------------------------------------- */
SW_API int32_t sw_version(void);                         /* 10000*major + 100*minor + patch */
/* The id of the sources this library was built from (16 hex digits of a
 * SHA-256 over csrc/ and include/, csrc/build_id.py); the Python binding
 * refuses a library whose id differs from the tree's (a stale build).     */
SW_API const char* sw_build_id(void);
SW_API const char* sw_last_error(void);                  /* thread-local text of the last failure */
SW_API int sw_encode(const char* ascii, int64_t n, uint8_t* codes);    /* SWSolver.cu:91-120 */
SW_API int sw_builtin_matrix(int32_t id, int8_t* out625);               /* SWSolver.cu:54-81 */

/* ---- device context ---------------------------------------------------
 * Replaces the reference's implicit CUDA context + default stream
 * (SWSolver.cu:282-288 allocations, :349/:381 synchronisations).        */
SW_API int sw_create(int32_t device, sw_handle** out);
SW_API int sw_destroy(sw_handle* h);
/* The handle's HIP stream (hipStream_t), e.g. to record events on it. */
SW_API void* sw_stream(sw_handle* h);
/* Use an external stream (e.g. torch's current stream); NULL = own stream. */
SW_API int sw_set_stream(sw_handle* h, void* hip_stream);

/* ---- kernel-form overrides ------------------------------------------------
 * The reference fixes every algorithm parameter at compile time (#defines,
 * SWSolver.cu:7,43-50).  This library chooses its kernel forms per scan from
 * the query, the database and the scoring; sw_opts overrides those choices
 * for tests and A/B measurements.  Scores never depend on it: every form is
 * bit-exact.  Every field is -1 (the library's own choice) after
 * sw_opts_init; a handle starts with those values.  The library reads no
 * environment variable on its scan path: sw_opts_from_env is the one place
 * the SW_* variables are read (test and measurement scripts call it).    */
typedef struct sw_opts {
    int32_t size;             /* sizeof(sw_opts), set by sw_opts_init (ABI check) */
    int32_t lpt;              /* 1: one merged longest-first launch (sw_scan_lpt)
                                 whenever the scan's shape allows it; 0: never  SW_LPT */
    int32_t lpt_pipe;         /* long-subject pairs the merged launch runs in the
                                 pipelined form (query chunk per wave)          SW_LPT_PIPE */
    int32_t quad_width;       /* inter blocks at least this wide run by wave quads
                                 in the merged launch (0: none)                SW_QUAD_WIDTH */
    int32_t pair_width;       /* ... by wave pairs (0: none)                   SW_PAIR_WIDTH */
    int32_t pair_group;       /* waves per group (2 or 4) of the separate pair
                                 launch                                        SW_PAIR_GROUP */
    int32_t coop_width;       /* blocks at least this wide go to the cooperative
                                 int32 kernel (int32 scans)                    SW_COOP_WIDTH */
    int32_t coop_skew;        /* 0: the cooperative kernel without its skew    SW_COOP_SKEW */
    int32_t intra_x2;         /* 0: long subjects in int32 only                SW_INTRA_X2 */
    int32_t intra_x2_rows;    /* rows per lane of the packed intra kernel
                                 (4, 6, 8, 10, 12, 16, 20)                     SW_INTRA_X2_RI */
    int32_t intra_i16_first;  /* 0 / 1: never / always run the long subjects'
                                 int16 form first (default: adaptive)          SW_INTRA_I16_FIRST */
    int32_t inter_i16_span;   /* the widest n blocks in int16 first (0: none;
                                 default: adaptive)                            SW_INTER_I16_SPAN */
    int32_t int16_guard;      /* 0: int32 beyond the static int16 bound        SW_INT16_GUARD */
    int32_t rescue_stats;     /* 1: print what the guard bands flagged per scan
                                 (synchronises)                                SW_RESCUE_STATS */
    int32_t tail_pairs;       /* the narrowest n blocks of the merged launch run
                                 by wave pairs (0: none)                       SW_TAIL_PAIRS */
    int32_t lpt_persist;      /* 0: the merged launch with one workgroup per work
                                 item, never one per resident slot taking items
                                 from a counter (default: that form for tables
                                 of 3+ rounds); n >= 2: that form with n
                                 workgroups (tests)                           SW_LPT_PERSIST */
    int32_t lpt_rows;         /* query rows per pass of the merged launch under
                                 linear gaps: 64 or 96 (default 96)           SW_LPT_ROWS */
    int32_t tri_width;        /* under affine gaps, the merged launch's widest group
                                 blocks at least this wide run by 3-wave groups
                                 (two rounds of a 6-pass query, no idle wave),
                                 whose workgroup's fourth wave runs a single-wave
                                 block, instead of quads (0: none; default
                                 0.48 x the long threshold on databases that run
                                 quads)                                      SW_TRI_WIDTH */
    int32_t lpt_pipe_tail;    /* the last n long-subject pairs of the merged
                                 launch (the shortest) run in the pipelined form
                                 too (0: none; default: 2 % of the pairs for
                                 linear scans of databases that run quads)   SW_LPT_PIPE_TAIL */
    int32_t drain_spin;       /* (tests) polls the merged launch's drain spends
                                 waiting for a claimed rescue-list entry before
                                 it gives up and faults (default 2^22; 0: at
                                 once, i.e. the SW_E_DEVICE path)             SW_DRAIN_SPIN */
    char inter_variant[16];   /* inter kernel shape: "" (auto), "32x8", "64x8"
                                 (int32), "y32x8" (int16 two-strips), "f32x8",
                                 "f32x4" (its fp16 form)                       SW_INTER_VARIANT */
    char trace_file[256];     /* per-workgroup timeline of the merged launch
                                 (builds with -DSW_TRACE_BLOCKS only; "" off)  SW_TRACE_FILE */
} sw_opts;
SW_API int sw_opts_init(sw_opts* o);
/* sw_opts_init, then every field whose SW_* variable (above) is set. */
SW_API int sw_opts_from_env(sw_opts* o);
SW_API int sw_set_opts(sw_handle* h, const sw_opts* o);
SW_API int sw_get_opts(const sw_handle* h, sw_opts* o);

/* ---- database -----------------------------------------------------------
 * Replaces the per-call packing loop SWSolver.cu:301-371 (longest-first
 * 32-lane interleave into managed memory, re-done on every query): the
 * database is sorted, packed and uploaded ONCE and stays resident in HBM.
 *   residues : encoded subject residues, concatenated
 *   offsets  : n+1 offsets into residues (offsets[0] = 0)
 *   ids      : n result ids (NULL = 0..n-1); sw_scan writes scores[id]   */
SW_API int sw_db_create(sw_handle* h, const uint8_t* residues, const int64_t* offsets,
                 int64_t n, const int32_t* ids, sw_db** out);
SW_API int sw_db_free(sw_db* db);
SW_API int sw_db_get_stats(const sw_db* db, sw_db_stats* out);
/* Binary database file (the intent of the reference's
 * parse.py:40-46): subjects sorted by length (descending, stable) as encoded
 * codes + int64 offsets + int32 result ids, with an FNV-1a checksum, so a
 * database is parsed from FASTA once and then loaded in one read.  Loading
 * gives a database whose scans produce identical scores[id].            */
SW_API int sw_db_save(const sw_db* db, const char* path);
SW_API int sw_db_load(sw_handle* h, const char* path, sw_db** out);
/* Synthetic database generated in HBM: subject
 * k (k = 0..n-1, result id k) has global id id_base + k; its length is
 * len4096[h(seed, gid, "LENGTH") >> 52] and residue j is
 * lut65536[(h(seed, gid, j >> 2) >> 16 (j & 3)) & 0xffff], with
 * h(seed, id, k) = mix(seed * 0x9E3779B97F4A7C15 + mix(id * 0xD6E8FEB86659FD93
 * + k)) and mix = splitmix64's finaliser (all mod 2^64).  Lengths are
 * log-normal (median 290, sigma 0.657, [5, 35213]), residues Swiss-Prot
 * frequencies.  Only O(n) metadata is computed on the host; the residues
 * are written by device kernels (no host copy, no PCIe transfer).  Any
 * subject can be regenerated on a CPU from the two tables (sw_synth_tables)
 * and the formula above, e.g. to check sampled scores.                  */
SW_API int sw_db_create_synthetic(sw_handle* h, uint64_t seed, int64_t id_base, int64_t n,
                                  sw_db** out);
SW_API int sw_synth_tables(int32_t* len4096, uint8_t* lut65536);
SW_API int sw_synth_lengths(uint64_t seed, int64_t id_base, int64_t n, int32_t* lengths);
/* Per-subject lengths and result ids in the database's order (the order of
 * sw_db_create's input, or of the file for sw_db_load); either may be NULL. */
SW_API int sw_db_subjects(const sw_db* db, int64_t* lengths, int32_t* ids);
/* Subjects longer than `threshold` go to the intra-sequence kernel (one
 * wave per subject) instead of the inter-sequence kernels (one subject per
 * lane).  0 = library default: 5.7 x the mean length clamped to
 * [1024, 8192]; from 64,000 to 570,000 subjects (a rank's share of a strong-
 * scaled database) scaled by (n / 570,000)^0.4, floor 512; 64 for databases
 * under 64,000 subjects with a mean length >= 256 (too few 64-subject blocks
 * to fill the GPU).  May be changed between scans (re-packs the database). */
SW_API int sw_db_set_long_threshold(sw_db* db, int32_t threshold);
/* A database learns from the flagged counts its scans read back (without
 * waiting) which work to run in int16 first: the widest blocks and the long
 * subjects, per scoring and query length (sw_opts inter_i16_span and
 * intra_i16_first override it).  Scores never depend on that state; which
 * kernels a scan runs does.  This forgets it (and any readback in flight),
 * so the next scan runs as on a fresh database: a caller can time a cold
 * and a warm scan deliberately.                                            */
SW_API int sw_db_reset_adaptive(sw_db* db);

/* ---- scans ---------------------------------------------------------------
 * Replaces smith_waterman_cuda (SWSolver.cu:266-404): score the encoded
 * query against every subject; scores[id] = best local score.  The output
 * array must hold max(id)+1 int32; slots no subject maps to are set to 0.
 * Synchronous.                                                            */
SW_API int sw_scan(sw_handle* h, const sw_db* db, const uint8_t* query, int32_t qlen,
            const sw_scoring* sc, int32_t* scores_host);

/* Same, asynchronous on the handle's stream, scores written to DEVICE memory
 * (scores_dev; only slots that some subject maps to are written).  Used by
 * bench.py with the database already resident.  The handle must outlive the
 * database: sw_db_free uses the handle's stream.                          */
SW_API int sw_scan_device(sw_handle* h, const sw_db* db, const uint8_t* query, int32_t qlen,
                   const sw_scoring* sc, int32_t* scores_dev);

/* Batch of nq queries (concatenated encoded residues, nq+1 offsets, query
 * k = queries[qoffsets[k] .. qoffsets[k+1])); scores_host is
 * [nq][max(id)+1].  The scans run back to back on the device with no host
 * synchronisation between queries (the reference's
 * main.cpp handles one query per run).  Synchronous.                      */
SW_API int sw_scan_batch(sw_handle* h, const sw_db* db, const uint8_t* queries,
                  const int64_t* qoffsets, int32_t nq, const sw_scoring* sc,
                  int32_t* scores_host);
/* Same, asynchronous on the handle's stream, into DEVICE memory scores_dev
 * [nq][max(id)+1] (only slots some subject maps to are written).          */
SW_API int sw_scan_batch_device(sw_handle* h, const sw_db* db, const uint8_t* queries,
                  const int64_t* qoffsets, int32_t nq, const sw_scoring* sc,
                  int32_t* scores_dev);

/* Timing of the most recent scan on this handle (waits for it). */
SW_API int sw_get_timing(sw_handle* h, sw_timing* out);
/* Kernel times summed over every scan since the last reset (waits for them);
 * *nscans = number of scans summed.  Lets a caller time many back-to-back
 * scans with HIP events on the stream they ran on, without synchronising
 * between them (bench.py).                                               */
SW_API int sw_timing_reset(sw_handle* h);
SW_API int sw_timing_total(sw_handle* h, sw_timing* out, int32_t* nscans);
/* Make another stream (hipStream_t, e.g. a top-K exchange stream) wait for
 * the handle's most recent scan to complete, through the scan's own end
 * event: no extra event record on the scan's stream (each is a packet the
 * command processor spends ~5 us on between two kernels).                 */
SW_API int sw_stream_wait_scan(sw_handle* h, void* hip_stream);
/* Name of the per-wave inter-sequence kernel the handle's last scan ran,
 * e.g. "sw_inter_x2<16,16,affine>" (packed int16, two subjects per lane) or
 * "sw_inter<32,8,affine>" (int32); "none" before any scan.  Valid until the
 * next scan on the handle.                                                  */
SW_API const char* sw_last_kernel(sw_handle* h);
/* Name of the intra-sequence (long-subject) kernel of the last scan:
 * "sw_intra_x2<16>" (two subjects per wave, packed fp16, with int32
 * re-scoring of flagged subjects), "sw_intra<6,affine>" (int32), or "none"
 * when the database has no long subjects.                                   */
SW_API const char* sw_last_intra_kernel(sw_handle* h);

/* ---- ranking ---------------------------------------------------------------
 * Top-k of a score vector (score descending, id ascending on ties).
 * Host-side helper for the multi-GPU top-K exchange.     */
SW_API int sw_topk(const int32_t* scores, int64_t n, int32_t k, int32_t* out_ids,
            int32_t* out_scores);

/* Device top-k, asynchronous on the handle's stream: the k best of
 * scores_dev[0..n) as int64 keys  score << 32 | (2^31 - 1 - (id_base + i)),
 * best first (score descending, id ascending); missing entries (n < k) are
 * INT64_MIN.  1 <= k <= 4096.  sw_topk_keys_device merges key vectors
 * (e.g. the all-gathered per-rank top-k of the multi-GPU exchange).        */
SW_API int sw_topk_device(sw_handle* h, const int32_t* scores_dev, int64_t n, int64_t id_base,
                   int32_t k, int64_t* keys_out_dev);
SW_API int sw_topk_keys_device(sw_handle* h, const int64_t* keys_dev, int64_t n, int32_t k,
                        int64_t* keys_out_dev);
/* A scan and its ranking in one synchronous call: the k best subjects of
 * the database for this query as int64 keys (sw_topk_device's: score << 32 |
 * 2^31 - 1 - result id, score descending, id ascending; INT64_MIN past the
 * database's end) in keys_host[k], from the device top-K over the scores of
 * every subject — only k keys cross PCIe.  The ranked output of main --topk
 * (the reference prints every score, main.cpp:58-60).  1 <= k <= 4096.    */
SW_API int sw_scan_topk(sw_handle* h, const sw_db* db, const uint8_t* query, int32_t qlen,
                        const sw_scoring* sc, int32_t k, int64_t* keys_host);
/* Same as sw_topk_device with the global id of entry i read from
 * ids_dev[i] (device int32, >= 0) instead of id_base + i: a rank's
 * residue-balanced shard of one database holds scattered
 * global ids, and the merged ranking breaks ties by global id.            */
SW_API int sw_topk_device_ids(sw_handle* h, const int32_t* scores_dev, int64_t n, const int32_t* ids_dev,
                              int32_t k, int64_t* keys_out_dev);
/* A scan and the ranking of its scores, asynchronous on the handle's stream:
 * sw_scan_device into scores_dev, then keys_out_dev[k] = the k best subjects
 * of the database as sw_topk_device keys (score << 32 | 2^31 - 1 - global id,
 * best first, INT64_MIN past the database's end), over the subjects' result
 * ids r, with global id gid_dev[r] (device int32, >= 0) or, gid_dev NULL,
 * id_base + r: main.cpp:54-60's scan-then-collect for one shard of the
 * multi-GPU search in one call.  The top-K launch follows
 * every stage that writes the scores and precedes the scan's end event
 * (sw_stream_wait_scan).  1 <= k <= 4096.                                   */
SW_API int sw_scan_rank_device(sw_handle* h, const sw_db* db, const uint8_t* query, int32_t qlen,
                               const sw_scoring* sc, int32_t* scores_dev, int32_t k, const int32_t* gid_dev,
                               int64_t id_base, int64_t* keys_out_dev);

/* ---- alignments of chosen hits (traceback) ------------------------------
 * The GPU analogue of the cpu.cpp pair program's traceback (cpu.cpp:47-108;
 * SURVEY.md §8 row f1): for each id in ids[0..n), the best local alignment of
 * the query against that database subject under cpu.cpp's rules — a cell
 * takes left, then up, then diagonal only on a strict improvement over 0,
 * the first strict maximum in row-major order is the end cell, and the walk
 * back stops at a zero cell.  Affine gaps (gap_open != gap_extend) use
 * this build's extension of those rules (the reference has no affine
 * traceback): a gap run opens unless extending is STRICTLY better, H takes
 * the run ending in the row (left), then the column (up), then the
 * diagonal, and the walk follows a run back to its opening cell; with
 * gap_open == gap_extend both give the same alignment.  Positions are
 * 1-based and inclusive; ops
 * (optional, n x ops_stride bytes, not NUL-terminated) spells the path from
 * the begin cell: 'M' an aligned pair, 'I' a query residue against a gap,
 * 'D' a subject residue against a gap; ops_len is the full path length even
 * when it exceeds ops_stride.  Cost O(|q| x |subject|) per hit: meant for
 * the top hits of a scan (e.g. the ids from sw_topk).                     */
typedef struct sw_alignment {
    int32_t score;
    int32_t q_begin, q_end;
    int32_t s_begin, s_end;
    int32_t ops_len;
} sw_alignment;
SW_API int sw_align(sw_handle* h, const sw_db* db, const uint8_t* query, int32_t qlen,
                    const sw_scoring* sc, const int32_t* ids, int32_t n, sw_alignment* out,
                    char* ops, int64_t ops_stride);

/* ---- single pair ---------------------------------------------------------
 * One query against one subject on the GPU (wavefront kernel); the GPU
 * analogue of the cpu.cpp pair program's score (cpu.cpp:43-74).         */
SW_API int sw_score_pair(sw_handle* h, const uint8_t* query, int32_t qlen,
                  const uint8_t* subject, int32_t slen, const sw_scoring* sc,
                  int32_t* score);

/* ---- several GPUs of one process -------------------------
 * Replaces the reference's single-GPU scan loop (main.cpp:54-56 ->
 * smith_waterman_cuda, SWSolver.cu:266-404) with one database sharded over
 * the devices of a group.  sw_group_create: one handle per listed device.
 * The first sw_group_topk of a group of DISTINCT devices creates an RCCL
 * communicator over them (ncclCommInitAll; librccl is loaded at run time,
 * only then: sw_group_scan needs no collective and no RCCL).  A device listed
 * twice is allowed (one-GPU tests), and RCCL that cannot be loaded or
 * initialised is tolerated: the top-K exchange then goes through the host.
 * sw_group_db_create: LPT shards over subject lengths (longest first, each to
 * the lightest shard, lowest index on ties: residue-balanced and
 * deterministic), one resident sw_db per device, built in parallel.
 * sw_group_scan: scores_host[id] of every subject (as sw_scan), the devices
 * scanning concurrently (one host thread each).  sw_group_topk: the k best
 * (score desc, id asc) as sw_topk_device keys in keys_host[k]: per-device
 * top-k with global ids, ONE ncclAllGather of k int64 keys per device, merge
 * on device 0.  All synchronous.                                          */
typedef struct sw_group sw_group;
typedef struct sw_gdb sw_gdb;
SW_API int sw_group_create(const int32_t* devices, int32_t ndev, sw_group** out);
SW_API int sw_group_destroy(sw_group* g);
/* The top-K exchange path: "rccl allgather (N ranks)" once the communicators
 * exist, "rccl allgather (communicators created by the first top-K)" before,
 * or "host (<why>)". */
SW_API const char* sw_group_info(const sw_group* g);
/* The handle of device slot d (owned by the group). */
SW_API int sw_group_handle(sw_group* g, int32_t d, sw_handle** out);
SW_API int sw_group_db_create(sw_group* g, const uint8_t* residues, const int64_t* offsets, int64_t n,
                              const int32_t* ids, sw_gdb** out);
SW_API int sw_group_db_free(sw_gdb* gdb);
/* Subjects and residues of shard d. */
SW_API int sw_group_db_shard(const sw_gdb* gdb, int32_t d, int64_t* n_subjects, int64_t* residues);
SW_API int sw_group_scan(sw_group* g, const sw_gdb* gdb, const uint8_t* query, int32_t qlen,
                         const sw_scoring* sc, int32_t* scores_host);
SW_API int sw_group_topk(sw_group* g, const sw_gdb* gdb, const uint8_t* query, int32_t qlen,
                         const sw_scoring* sc, int32_t k, int64_t* keys_host);

#ifdef __cplusplus
}
#endif
#endif /* SW_AMD_H */
