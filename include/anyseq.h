/*
 * anyseq.h — C-ABI of the MI355X-native AnySeq engine (libanyseq.so).
 *
 * The first block is exactly the reference's FFI for the hot path:
 *   /root/reference/src/import.h:14-41 (+ datatypes.h:14 score_t = int64_t),
 * defined there by export.impala:5-166.  The reference's own driver
 * (src/main.cpp, sequence_io.cpp, alignment_io.cpp) compiles unchanged against
 * this header and links against libanyseq.so.
 *
 * Fixed scoring for these six: match +2, mismatch -1, linear gap -1
 * (linear_scoring_scheme(2,-1,-1), export.impala:14,33,70,89,126,145).
 *
 * Semantics (bit-exact with the reference CPU path, iteration_cpu/scoring_cpu,
 * with `benchmark` running its body once — SURVEY.md §0.1):
 *   *_score       optimal score: global H[n-1][m-1]; semiglobal max over the last
 *                 row/column incl. the zero border; local max cell (an empty
 *                 sequence gives -2147483647, the never-written slot value).
 *   construct_*   alQuery/alSubject (caller-allocated, >= lenq+lens bytes each)
 *                 receive the reference's sparse layout: [0, lenq+lens) first set
 *                 to ' ', then each traceback step writes at i+j+1, gaps are '_'
 *                 (traceback.impala:14-80), no NUL written.  The strings come from
 *                 the reference's column-split Hirschberg (align.impala:237-311).
 *                 Return value: the reference's literal value (-lenq / 0 /
 *                 -2147483647) unless ANYSEQ_CONSTRUCT_TRUE_SCORE=1
 *                 is set in the environment, in which case the optimal score.
 * Errors: on an internal GPU failure these return INT64_MIN and print to stderr;
 * anyseq_last_error() holds the message.
 */
#ifndef ANYSEQ_H_
#define ANYSEQ_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- reference ABI: import.h:14-27 ---- */
int64_t construct_global_alignment(const char* query, int lenq, const char* subject, int lens, char* alQuery,
                                   char* alSubject);
int64_t construct_semiglobal_alignment(const char* query, int lenq, const char* subject, int lens, char* alQuery,
                                       char* alSubject);
int64_t construct_local_alignment(const char* query, int lenq, const char* subject, int lens, char* alQuery,
                                  char* alSubject);

/* ---- reference ABI: import.h:31-41 ---- */
int64_t global_alignment_score(const char* query, int lenq, const char* subject, int lens);
int64_t semiglobal_alignment_score(const char* query, int lenq, const char* subject, int lens);
int64_t local_alignment_score(const char* query, int lenq, const char* subject, int lens);

/* ---- reference exports not declared in import.h: export.impala:37-53, 93-109,
 * 150-166.  Full-matrix traceback (traceback_full, align.impala:190-216): every
 * predecessor of the n x m matrix, walked from (n-1, m-1).  As in the reference,
 * ALL THREE use the global scheme (export.impala:52,108,165).  Same sparse output
 * layout as construct_*; returns H[n-1][m-1].  Memory O(n*m) (limit 16 GB). ---- */
int64_t construct_global_alignment_fulltb(const char* query, int lenq, const char* subject, int lens, char* alQuery,
                                          char* alSubject);
int64_t construct_semiglobal_alignment_fulltb(const char* query, int lenq, const char* subject, int lens,
                                              char* alQuery, char* alSubject);
int64_t construct_local_alignment_fulltb(const char* query, int lenq, const char* subject, int lens, char* alQuery,
                                         char* alSubject);

/* ---- extended API (build-defined; not part of the reference) ---- */
enum { ANYSEQ_GLOBAL = 0, ANYSEQ_SEMIGLOBAL = 1, ANYSEQ_LOCAL = 2 };

/* Scoring: substitution match/mismatch; a gap of length k costs gap_open + k*gap_extend.
 * gap_open == 0 is the reference's linear scheme (gap = gap_extend).  Requires
 * gap_extend < 0 and gap_open <= 0. */
typedef struct {
    int32_t match, mismatch, gap_open, gap_extend;
} anyseq_scoring;

/* Host buffers in, optimal score out.  Returns 0 on success, <0 on error. */
int anyseq_score(int kind, const anyseq_scoring* sc, const char* query, int lenq, const char* subject, int lens,
                 int64_t* score);

/* Device-resident inputs (d_query/d_subject are device pointers of the current
 * device); runs on `stream` (hipStream_t, NULL = the engine's own stream) and
 * returns after the score has been copied back. */
int anyseq_score_device(int kind, const anyseq_scoring* sc, const uint8_t* d_query, int lenq, const uint8_t* d_subject,
                        int lens, void* stream, int64_t* score);

/* Linear-space alignment with the reference's column-split Hirschberg, sparse
 * i+j+1 layout as construct_*; *score (optional) receives the optimal score. */
int anyseq_construct(int kind, const anyseq_scoring* sc, const char* query, int lenq, const char* subject, int lens,
                     char* alQuery, char* alSubject, int64_t* score);

/* anyseq_construct on device-resident sequences (device pointers of the current
 * device) into device strings d_alQuery/d_alSubject of lenq+lens bytes each; runs
 * on `stream` (NULL = the engine's own) and returns when the strings are complete. */
int anyseq_construct_device(int kind, const anyseq_scoring* sc, const uint8_t* d_query, int lenq,
                            const uint8_t* d_subject, int lens, uint8_t* d_alQuery, uint8_t* d_alSubject, void* stream,
                            int64_t* score);

/* Device selection (default: $ANYSEQ_DEVICE or 0) and diagnostics. */
int anyseq_set_device(int device);
int anyseq_get_device(void);
const char* anyseq_last_error(void);

/* Fill-kernel tuning: rows per lane (1,2,4), compute waves per workgroup (3,4,7,8),
 * persistent grid size (0 = one workgroup per CU).  0 keeps the current value. */
void anyseq_set_tuning(int rows_per_lane, int waves_per_group, int grid);

/* Named tuning option: "rows_per_lane" (1,2,4), "chunk" (16,32 steps per block),
 * "waves_per_group" (3,4,7,8), "grid", "fronts" (1 or 2: score fill as one
 * front or two meeting fronts), "affine_waves_per_group" (3,4,7,8),
 * "affine_rows_per_lane" (0,1,2,3), "affine_self_forward", "linear_via_affine",
 * "affine_grid", "ring_slots" (group hand-off rows kept per sub-problem; 0 = 4*grid+4,
 * never fewer than 2*grid+2), and the others INTEGRATION.md lists.
 * Returns 0, or -1 for an unknown name. */
int anyseq_set_option(const char* name, int value);

/* Timing of the most recent fill launch(es) of the calling thread, measured with
 * HIP events on the engine stream: total kernel milliseconds and launch count. */
void anyseq_last_fill_timing(double* ms, int* launches);
/* The same, plus the DP cells those launches computed (sum of h*w of their
 * sub-problems).  Both reset the counters. */
void anyseq_last_fill_stats(double* ms, int* launches, int64_t* cells);
/* Plan of the calling thread's most recent sharded construct (anyseq_shard_construct,
 * anyseq_construct_local_sharded): the number of leading Hirschberg levels whose
 * halves were column-blocked over rank subgroups (level 1 over all ranks; 0: every
 * level dealt round-robin, e.g. when GPU_MAX_HW_QUEUES is too small for the concurrent
 * shard streams).  Resets it. */
int anyseq_last_shard_plan(void);
/* Affine fill launches of the calling thread since the previous call that ran two or three
 * rows per lane (64 R-row bands; chosen per launch or by the option
 * "affine_rows_per_lane"); *max_rows (may be null) gets the most rows per lane among the
 * launches (1 when none).  Resets both. */
int anyseq_last_fill_multi_row_launches(int* max_rows);
/* Affine construct, host-built levels (option "inherit_halves"): the
 * halves of the calling thread's constructs since the previous call that ran as two column
 * blocks recording their child's column (the return value), and the halves taken as such a
 * recorded column instead of a fill (*reused, may be null).  Resets both. */
int64_t anyseq_last_inherit_stats(int64_t* reused);

/* ---- column-block sharded score (build-defined) ----
 * Subject columns are split into contiguous blocks, block g = [g*m/N, (g+1)*m/N);
 * the boundary columns of the two fill fronts travel between neighbouring shards
 * in row chunks while the fills run.  Linear and affine gaps (affine: the column
 * carries H and E, plus F of the front's last row).
 *
 * One process per GPU over RCCL: rank 0 calls anyseq_shard_unique_ids (count = 4),
 * the bytes (count * 128) are broadcast out of band, every rank calls
 * anyseq_shard_init, anyseq_shard_load (its block), then anyseq_shard_score
 * (collective; every rank receives the full score). */
int anyseq_shard_unique_ids(void* ids, int count);
int anyseq_shard_init(int rank, int world, const void* ids, int count);
int anyseq_shard_load(const char* query, int lenq, const char* subject_block, int block_len, int block_offset,
                      int lens);
int anyseq_shard_score(int kind, const anyseq_scoring* sc, int64_t* score);
int anyseq_shard_finalize(void);
/* The same sharded fill with `nshards` shards inside this process on the current
 * device (device copies instead of RCCL between them). */
/* Sharded affine construct (align.impala:237-311 distributed by level):
 * every rank calls it with the whole pair after anyseq_shard_init.  Level 1's two
 * halves are column-blocked over ALL ranks (rank g fills query columns
 * [g*lenq/N, (g+1)*lenq/N) of both, boundary columns over RCCL send/recv); every later
 * level with P parts and N >= 2P ranks is column-blocked the same way, part p over the
 * rank subgroup [p*N/P, (p+1)*N/P); the half fills of the remaining levels and the final
 * 128-column blocks are dealt round-robin; the level columns are all-reduced over RCCL,
 * and every rank returns the same score and strings (sparse i+j+1 layout, lenq+lens
 * bytes each).  When GPU_MAX_HW_QUEUES leaves too few hardware queues for the concurrent
 * transport streams, those levels are dealt round-robin too (same result;
 * anyseq_last_shard_plan reports which plan ran). */
int anyseq_shard_construct(int kind, const anyseq_scoring* sc, const char* query, int lenq, const char* subject,
                           int lens, char* alQuery, char* alSubject, int64_t* score);
/* The same plan with `nshards` virtual ranks in this process on one device (one fill
 * launch per rank per level): the 1-GPU parity check of the sharded construct.  Its
 * column-blocked level 1 needs 3*nshards-2 streams and nshards co-resident grids
 * (nshards <= CUs/8 - 8); otherwise level 1 is dealt round-robin. */
int anyseq_construct_local_sharded(int kind, const anyseq_scoring* sc, const char* query, int lenq,
                                   const char* subject, int lens, int nshards, char* alQuery, char* alSubject,
                                   int64_t* score);
int anyseq_shard_score_local(int kind, const anyseq_scoring* sc, const char* query, int lenq, const char* subject,
                             int lens, int nshards, int64_t* score);
/* The one-rank-per-process plan of anyseq_shard_construct (this process is `rank` of
 * `world`: it fills only its own halves and final blocks), with the level reductions
 * through a host callback instead of RCCL: `reduce(buf, count, dtype, op, user)` must
 * all-reduce `count` elements of the host buffer in place over the ranks (dtype 0 int32,
 * 1 uint8; op 0 SUM, 1 MAX) and return 0.  No column-blocked levels (they need the
 * send/recv transport): every level is dealt round-robin.  Test transport: it runs the
 * rank >= 0 branch of the sharded construct (several processes may share one device,
 * which RCCL refuses) against the single-GPU construct. */
typedef int (*anyseq_host_allreduce_fn)(void* buf, int64_t count, int dtype, int op, void* user);
int anyseq_shard_construct_hostcoll(int kind, const anyseq_scoring* sc, const char* query, int lenq,
                                    const char* subject, int lens, int rank, int world,
                                    anyseq_host_allreduce_fn reduce, void* user, char* alQuery, char* alSubject,
                                    int64_t* score);

/* ---- alignment-output adapters (host only) ----
 * The sparse i+j+1 layout of construct_* / anyseq_construct (len = lenq+lens):
 * anyseq_alignment_dense drops the positions blank in both strings and writes the
 * dense pair (either output may be NULL); returns its length.
 * anyseq_alignment_cigar writes the extended CIGAR (=, X, I, D; '_' in alQuery ->
 * D, '_' in alSubject -> I) NUL-terminated into out (at most cap bytes, truncated
 * like snprintf) and returns its full length; out may be NULL to size it.
 * Both return -1 on invalid arguments. */
int64_t anyseq_alignment_dense(const char* alQuery, const char* alSubject, int64_t len, char* outQuery,
                               char* outSubject);
int64_t anyseq_alignment_cigar(const char* alQuery, const char* alSubject, int64_t len, char* out, int64_t cap);

/* main.cpp's random input generator (main.cpp:90-120, 200-210): mt19937_64 with the
 * default seed, lengths uniform in [minlen, maxlen], bases uniform over ACGT.
 * query/subject must hold maxlen bytes; lengths are returned. */
void anyseq_main_random_pair(int64_t minlen, int64_t maxlen, char* query, int64_t* lenq, char* subject,
                             int64_t* lens);

#ifdef __cplusplus
}
#endif

#endif /* ANYSEQ_H_ */
