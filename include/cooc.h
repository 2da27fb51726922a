/*
 * cooc.h — C-ABI of the MI355X co-occurrence core (pair expansion + keyed (itemA,itemB) count
 * reduction, the non-sampled path of uce/flink-cooccurrence).
 *
 * Boundary.  The entry points replace, for the `--skip-cuts` job graph of
 * FlinkCooccurrences.java:65-74,135-167, everything between the keyBy(user) edge and the sink:
 *
 *   reference (file:line, under src/main/java/com/github/uce/flinkcooccurrences/)   replaced by
 *   ------------------------------------------------------------------------------  -------------------------------
 *   NonSampledUserInteractionCounterOneInputStreamOperator.processElement :84-110   cooc_op_process_elements
 *   NonSampledUserInteractionCounterOneInputStreamOperator.onEventTime    :113-165  cooc_op_process_watermark /
 *     (+ ItemCooccurrences record & Kryo codec, ItemCooccurrences.java:14-149)        cooc_submit_batch +
 *   ItemRowAggregator.ItemCooccurrenceRowAggregateFunction.add            :26-31      cooc_finish_window
 *   ItemRowAggregator.ItemCooccurrenceRowWindowFunction.process           :50-56    cooc_copy_window_delta
 *   RowSumAggregator.RowSumAggregateFunction.add / RowSumProcessWindow    :25-71    cooc_copy_window_rowsums
 *   ItemRowRescorerTwoInputStreamOperator.processWatermark..scoreItem     :116-241  cooc_copy_window_topk
 *   LogLikelihood.logLikelihoodRatio                                       :41-57    (inside the rescoring kernel)
 *   IntDoublePriorityQueue add/update/iterator                             :132-242  (heap layout of topk output)
 *   UserInteractionCounterObservedCooccurrences / LateElements /
 *   RowSumProcessWindowRowSum / ItemRowRescorerRescoredItems accumulators            cooc_op_counters
 *
 * plus one stateless entry point over a device-resident CSR of user histories
 * (cooc_count_device): one tumbling window over empty histories, the unit the benchmark times.
 *
 * Conventions:
 *  - Every function returns an int status (COOC_OK = 0); the message of the last failure on a
 *    context is cooc_last_error(ctx).  The Java wrapper rethrows IllegalStateException /
 *    IllegalArgumentException where the reference throws them.
 *  - The library never retains caller pointers after a call returns.  Results are either copied
 *    into caller buffers (two-phase: sizes from cooc_window_info, then cooc_copy_*), or handed
 *    out as BORROWED device views that stay valid until the next call on the same context.
 *  - One context per Flink subtask; a context is not thread-safe, distinct contexts are.
 *  - Item ids must lie in [0, cfg.n_items); user ids are arbitrary int32 (keyed state).
 *  - Counts are exact (uint32, overflow is detected and reported as COOC_ERR_OVERFLOW); the
 *    reference's own int16 (Int2ShortOpenHashMap) and int32 (Int2IntOpenHashMap / IntValue) wrapped
 *    views are produced by the copy functions ("ref_compat").
 *  - There is no CPU fallback: without a usable HIP device every compute entry point fails with
 *    COOC_ERR_HIP.
 *  - Streams.  An entry point that takes device pointers and a `hip_stream` runs its kernels on that
 *    stream; NULL is the HIP null stream (which orders with hipMemcpy and with torch's default
 *    stream).  The caller must have ENQUEUED the work producing the inputs on the same stream (or
 *    ordered it before, e.g. with an event); the library never reads caller buffers from another
 *    stream.  Entry points that return host values (sizes, counts) synchronise that stream first.
 *  - No C++ exception crosses this boundary: host allocation failures return COOC_ERR_OOM, any
 *    other internal exception COOC_ERR_STATE, with the message in cooc_last_error.
 */
#ifndef COOC_H_
#define COOC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define COOC_ABI_VERSION 7

#if defined(__GNUC__)
#define COOC_API __attribute__((visibility("default")))
#else
#define COOC_API
#endif

enum cooc_status {
  COOC_OK = 0,
  COOC_ERR_ARG = 1,      /* IllegalArgumentException in the reference */
  COOC_ERR_STATE = 2,    /* IllegalStateException in the reference */
  COOC_ERR_HIP = 3,      /* HIP runtime / no device */
  COOC_ERR_OOM = 4,      /* device allocation failed */
  COOC_ERR_OVERFLOW = 5  /* an exact uint32 count overflowed */
};

/* cooc_config.flags. */
#define COOC_FLAG_EXACT_SCORES 1 /* LLR on exact counts instead of the reference's wrapped int16/int32 */
/* Layout of a cooc_count_device result (default: automatic, dense when the ordered pairs cover at
 * least half of the n_items^2 matrix and it fits in HBM, else the padded CSR). */
#define COOC_FLAG_OUTPUT_CSR 2   /* always the padded CSR (row_base, row_nnz, col, cnt) */
#define COOC_FLAG_OUTPUT_DENSE 4 /* always the dense matrix (dense, row_nnz) */
/* Route every window through the large-universe planner (the path for n_items >= 40,320: per-row LDS
 * hash / dense-tile chunks) even when the batch planner applies; same results (A/B and tests). */
#define COOC_FLAG_GENERAL_PLANNER 8
/* Large universes: every whole row through the sort + segmented-reduce path (packed 64-bit (row, column)
 * pair keys, radix-sorted, runs counted) instead of the LDS hash / dense-tile chunks.  That path always
 * takes the rows whose LDS hash table overflows; the flag sends all of them (A/B and tests). */
#define COOC_FLAG_SORT_ROWS 16
/* Large universes, batch windows: keep the columns of a row in ascending id order.  By default the
 * large-universe path renumbers the columns of a batch so that its first 16,384-column tile holds the
 * batch's 16,384 most frequent items (that batch's item counts, or the global counts of
 * cooc_count_device_owned): column c < 16,384 is the c-th of those hot items in ASCENDING id order, and
 * every other item b is column b + 16,384 (the hot items leave holes there).  The renumbering is skipped
 * -- identity order -- when at least 15/16 of the hot items already have ids below 16,384 (ids numbered by
 * popularity), and for universes of one tile.  A device result's rows are in this column order, which is
 * also the order the rescorer scores them in (the top-k tie order); cooc_copy_column_order reports it.
 * The host copies (cooc_copy_batch) are always in ascending id order.  This flag keeps id order on the
 * device at the price of the renumbering's gain (ids not numbered by popularity run up to ~1.8x slower). */
#define COOC_FLAG_COLUMN_ORDER 32
/* Large universes, batch results: a row's entries may come out in any order (the row holds the same keys and
 * counts).  Without it every row is in the result's column order, which costs the LDS hash chunks a column
 * ranking of their keys; the reference's own row is an Int2ShortOpenHashMap, iterated in slot order
 * (ItemRowAggregator.java:50-56, ItemRowRescorer...java:195), so a consumer that builds maps from the rows
 * (the Flink rows operators) or only sums them needs no order.  The host copies (cooc_copy_batch,
 * cooc_copy_batch_range) still sort every row; the top-k of an unordered result feeds each heap in the row's
 * order (ties may resolve differently, as between two fastutil builds); cooc_verify_batch checks keys,
 * counts and sums but not the order (and not the symmetry: [5] = -1); cooc_partition_plan refuses such a
 * result (the partial-row merge needs ordered rows).  Streaming windows always keep column order. */
#define COOC_FLAG_ANY_ORDER 64

typedef struct cooc_ctx cooc_ctx;

typedef struct cooc_config {
  int32_t device;         /* HIP device ordinal; -1 = the current device */
  int32_t n_items;        /* item-id universe: ids in [0, n_items) */
  int32_t topk;           /* ItemRowRescorer topK (ItemRowRescorer...java:51-56, Configuration.java:153);
                             0 disables rescoring */
  int32_t flags;          /* COOC_FLAG_* */
  int64_t window_size_ms; /* TumblingEventTimeWindows.of(Time.of(windowSize, windowUnit)),
                             NonSampled...java:61-62, in milliseconds */
  int32_t user_cut;       /* kMax: 0 = off (the non-sampled path).  1..32767 (a Java short,
                             UserInteractionCounter...java:54,76): only the first user_cut
                             interactions of every user (arrival order, over all windows) are
                             expanded -- the `userInteractions < userCut` branch of
                             UserInteractionCounter...java:168-205; later interactions are dropped
                             (the reference's random reservoir branch, :206-240, is not restated) */
  int32_t reserved;
} cooc_config;

/* Sizes of one fired window's outputs (two-phase copy protocol). */
typedef struct cooc_window_info {
  int64_t ts;             /* window.maxTimestamp(): timestamp of every output record, NonSampled...java:115 */
  int64_t nnz;            /* entries over all delta rows */
  int64_t observed;       /* exact ordered pairs of the window: sum of 2*|history| (NonSampled...java:153) */
  int32_t n_rows;         /* items with a delta row (= items with a row-sum update) */
  int32_t topk;           /* columns of the top-k output (cfg.topk) */
  int32_t n_topk;         /* rescored rows (n_rows when topk > 0, else 0) */
  int32_t reserved;
} cooc_window_info;

/* Borrowed device views of a cooc_count_device result (valid until the next call on ctx).  Exactly
 * one layout is set: the padded CSR (row_base, col, cnt non-NULL, dense NULL) or the dense matrix
 * (dense non-NULL, row_base / col / cnt NULL).  Both key sets are the reference's touched keys: a
 * key exists iff its count is > 0 (every increment is +1, ItemRowAggregator.java:29). */
typedef struct cooc_device_result {
  int64_t n_items;
  int64_t nnz;            /* total entries (keys with a count > 0) */
  int64_t observed;       /* exact ordered pairs sum_u n_u (n_u - 1) */
  const int64_t *row_base;  /* [n_items]: first entry of row a in col/cnt (rows padded, not packed) */
  const int32_t *row_nnz;   /* [n_items]: entries of row a (both layouts) */
  const int32_t *col;       /* item ids, ascending within a row in the result's column order: the id itself,
                               or, for a renumbered large-universe batch (n_items >= 40,320 without
                               COOC_FLAG_COLUMN_ORDER), the hot items first in id order, then the others in
                               id order (see COOC_FLAG_COLUMN_ORDER, cooc_copy_column_order) */
  const uint32_t *cnt;      /* exact counts */
  const int64_t *rowsum;    /* [n_items]: exact row sums sum_b C[a,b] */
  const uint32_t *dense;    /* [n_items * n_items] row-major exact counts, 0 = key absent */
} cooc_device_result;

/* ---- lifecycle ------------------------------------------------------------------------------ */
COOC_API int cooc_abi_version(void);
COOC_API const char *cooc_status_string(int status);
COOC_API int cooc_create(const cooc_config *cfg, cooc_ctx **out);
/* create(cfg{devices[]}) of SURVEY §8(b): one handle per Flink subtask over the node's GPUs.  The
 * handle binds to devices[subtask % n_devices] (cfg->device is ignored); every other field as in
 * cooc_create.  A device ordinal outside [0, hipGetDeviceCount()) is COOC_ERR_ARG. */
COOC_API int cooc_create_on(const cooc_config *cfg, const int32_t *devices, int32_t n_devices, int32_t subtask,
                            cooc_ctx **out);
COOC_API void cooc_destroy(cooc_ctx *ctx);
COOC_API const char *cooc_last_error(const cooc_ctx *ctx);

/* ---- stateless one-window batch over a device CSR (the benchmarked unit) ----------------------
 * d_user_ptr: int64[n_users+1] offsets into d_items (device memory); d_items: int32[n_interactions]
 * in per-user arrival order.  hip_stream: a hipStream_t (NULL = the HIP null stream).
 * Computes C = sum over users of the ordered position pairs (p != q) -> (x_p, x_q), i.e. exactly
 * what NonSampled...java:113-165 emits for users whose histories start empty, reduced by
 * ItemRowAggregator/RowSumAggregator.  Does not touch the context's streaming state. */
COOC_API int cooc_count_device(cooc_ctx *ctx, int64_t n_users, const int64_t *d_user_ptr, const int32_t *d_items,
                      int64_t n_interactions, void *hip_stream, cooc_device_result *out);
/* Multi-GPU for large item universes (n_items >= 40,320, the C3 / C5 configs): the keyBy(itemA) of
 * FlinkCooccurrences.java:152 as row ownership.  Counts only the rows a with d_owner[a] == part, over
 * every user given (the all-gathered log of all parts); rows owned by other parts come out empty.
 * d_item_counts int64[n_items]: the global log's item frequencies (n_total interactions in all),
 * which size the planner; out->observed = the ordered pairs of the owned rows (their sum over the
 * parts is the log's sum_u n_u (n_u - 1)).  Same borrowed padded-CSR result as cooc_count_device. */
COOC_API int cooc_count_device_owned(cooc_ctx *ctx, int64_t n_users, const int64_t *d_user_ptr, const int32_t *d_items,
                                     int64_t n_interactions, const int32_t *d_owner, int32_t part,
                                     const int64_t *d_item_counts, int64_t n_total, void *hip_stream,
                                     cooc_device_result *out);
/* Item frequencies of a device item array (d_items int32[n_interactions]) into d_counts int64[n_items]
 * (device, overwritten) on hip_stream: the local part of the global frequencies that
 * cooc_count_device_owned's caller all-reduces (owner map, planner estimate).  Ids outside
 * [0, n_items) are not counted.  Each workgroup counts the items it meets most in an LDS table (the
 * Zipf head, whatever its ids) and sends the rest to global 64-bit atomics. */
COOC_API int cooc_item_counts(cooc_ctx *ctx, const int32_t *d_items, int64_t n_interactions, int64_t *d_counts,
                              void *hip_stream);
/* The column order of the last batch result's device rows (and of its top-k iteration, the tie order):
 * rank_of int32[n_items] gets the position of every item in that order -- after a large-universe
 * renumbering, c for the c-th hot item (ascending ids) and id + 16,384 for every other item; else the id
 * itself (see COOC_FLAG_COLUMN_ORDER for when the renumbering happens).  Only the relative order counts. */
COOC_API int cooc_copy_column_order(cooc_ctx *ctx, int32_t *rank_of);
/* Same from host buffers; afterwards cooc_copy_batch copies the packed CSR out. */
COOC_API int cooc_count_host(cooc_ctx *ctx, int64_t n_users, const int64_t *user_ptr, const int32_t *items,
                    cooc_window_info *info);
/* Packed CSR over ALL n_items rows: row_ptr int64[n_items+1]; cols/cnt/cnt16 [nnz];
 * rowsum int64[n_items], rowsum32 int32[n_items].  Any pointer may be NULL. */
COOC_API int cooc_copy_batch(cooc_ctx *ctx, int64_t *row_ptr, int32_t *cols, uint32_t *cnt, int16_t *cnt16, int64_t *rowsum,
                    int32_t *rowsum32);

/* The entries of batch rows [row_begin, row_end) only, in cooc_copy_batch's packed order (row_ptr from a
 * cooc_copy_batch call with cols/cnt/cnt16 NULL): cols/cnt/cnt16 hold at least `cap` entries; a range of more
 * entries than cap is COOC_ERR_ARG and nothing is written.  A JVM operator streams a result larger than one
 * Java array (a C3 share: ~7e9 entries; an owner's rows: ~4e9) out in row ranges (ItemRowAggregator.java:50-56's
 * one map per row).  The packed view is built once per batch. */
COOC_API int cooc_copy_batch_range(cooc_ctx *ctx, int32_t row_begin, int32_t row_end, int64_t cap, int32_t *cols,
                                   uint32_t *cnt, int16_t *cnt16);
/* LLR top-k of every row of the last cooc_count_device / cooc_count_host result: what
 * ItemRowRescorer...java:195-241 emits after that one window from an empty state (rows iterated in
 * ascending column order, LogLikelihood.java:41-57 scores, IntDoublePriorityQueue layout).  flags:
 * COOC_FLAG_EXACT_SCORES to score exact counts instead of the reference's wrapped int16/int32.
 * cooc_copy_topk_batch: sizes int32[n_items], values int32[n_items*topk], scores double[n_items*topk]
 * (heap positions 1..size, least score first; rows without entries have size 0). */
/* hip_stream NULL = the context's own stream (no caller stream is kept between calls: the count this
 * scores has drained before cooc_count_device returned, and cooc_topk_batch synchronises the stream it
 * runs on before returning). */
COOC_API int cooc_topk_batch(cooc_ctx *ctx, int32_t topk, int32_t flags, void *hip_stream);
COOC_API int cooc_copy_topk_batch(cooc_ctx *ctx, int32_t *sizes, int32_t *values, double *scores);
/* The same top-k into caller DEVICE buffers on hip_stream (ordered after the count on the caller's
 * stream; the C5 config keeps its output resident): d_sizes int32[n_items], d_values
 * int32[n_items*topk], d_scores double[n_items*topk].  d_rowsum_global (device int64[n_items], may be
 * NULL) replaces the result's own row sums: multi-GPU owners pass the all-reduced row sums (the
 * broadcast row-sum stream, FlinkCooccurrences.java:163), so that k21 = rowSum(b) - k11 and the
 * observed total (ItemRowRescorer...java:154,203-240) are the whole log's; rows the context does not
 * own have no entries and get size 0. */
COOC_API int cooc_topk_batch_device(cooc_ctx *ctx, int32_t topk, int32_t flags, const int64_t *d_rowsum_global,
                                    int32_t *d_sizes, int32_t *d_values, double *d_scores, void *hip_stream);
/* LogLikelihood.logLikelihoodRatio (LogLikelihood.java:41-57) evaluated by the device function the
 * rescoring kernels use: k = host int64[n][4] of (k11, k12, k21, k22), out = host double[n].  For
 * known-answer tests of the device scores (LogLikelihoodTest.java:14-16). */
COOC_API int cooc_llr(cooc_ctx *ctx, int64_t n, const int64_t *k, double *out);
/* The SURVEY §8(b) query topk(handle, items[], k): the top-k of the rows `items` (n of them) of the
 * last batch result, computing the batch top-k first when it has not run with this (k, flags).
 * out_sizes int32[n], out_items int32[n*k], out_scores double[n*k] (heap positions 1..size as in
 * cooc_copy_topk_batch).  The rescorer's per-row query (ItemRowRescorer...java:195-241 for the
 * given rows only); an item outside [0, n_items) is COOC_ERR_ARG. */
COOC_API int cooc_topk_items(cooc_ctx *ctx, int32_t k, int32_t flags, int32_t n, const int32_t *items,
                             int32_t *out_sizes, int32_t *out_items, double *out_scores);

/* ---- streaming (resident per-user histories, global rows, row sums) ------------------------
 * cooc_submit_batch stages the interactions of one tumbling window: n_users users with their
 * new items in arrival order (user_ptr int64[n_users+1] into items).  Several submits to the same
 * window append.  cooc_finish_window expands every staged user against its resident history,
 * reduces the window's delta rows and row sums, merges them into the global state and, if
 * topk > 0, rescores every touched row (ItemRowRescorer...java:144-228).
 * Across GPUs (a communicator of world > 1 on ctx, cooc_comm_init / cooc_comm_init_ops; any item universe: below
 * 40,320 items the owners keep dense global rows, above it sorted row slabs): each context holds the resident histories of ITS users (a keyBy(user) shard,
 * FlinkCooccurrences.java:70) and cooc_finish_window is collective: every rank expands its own users, the
 * partial delta rows go to their owners (row a on rank a mod world: the keyBy(item) of :152), the row-sum
 * deltas and the window's pairs are all-reduced (the broadcast of :163), and each owner merges its rows into
 * its resident global rows and rescores them against the job's row sums.  The window's outputs on a rank
 * are its owned rows (every row of the job on exactly one rank); info->observed is this rank's users' pairs
 * (the ObservedCooccurrences accumulator; the ranks' values add up to the job's).  Every rank finishes the
 * same windows in the same order: cooc_op_process_watermark decides from all-gathered state only (the ranks'
 * watermarks and earliest pending windows), so ranks that receive different watermark sequences still run the
 * same collectives, and a rank without records in a window still joins it. */
COOC_API int cooc_submit_batch(cooc_ctx *ctx, int64_t window_ts, int32_t n_users, const int32_t *user_ids,
                      const int64_t *user_ptr, const int32_t *items);
COOC_API int cooc_finish_window(cooc_ctx *ctx, int64_t window_ts, cooc_window_info *info);

/* Delta rows of the last finished window (ItemCooccurrenceRowWindowFunction output):
 * rows int32[n_rows] ascending, row_ptr int64[n_rows+1], cols/cnt/cnt16 [nnz].  NULLs skipped. */
COOC_API int cooc_copy_window_delta(cooc_ctx *ctx, int32_t *rows, int64_t *row_ptr, int32_t *cols, uint32_t *cnt,
                           int16_t *cnt16);
/* The entries of delta rows [row_begin, row_end) only (row indices as in cooc_copy_window_delta's rows[]):
 * cols/cnt/cnt16 [row_ptr[row_end] - row_ptr[row_begin]], each holding at least `cap` entries: a range of
 * more entries than cap is COOC_ERR_ARG and nothing is written.  A window whose delta holds more entries than
 * one Java array can (2^31 - 1) streams out in row ranges: first cooc_copy_window_delta(rows, row_ptr,
 * NULL, NULL, NULL), then ranges sized from row_ptr.  The packed copy-out view is built once per window. */
COOC_API int cooc_copy_window_delta_range(cooc_ctx *ctx, int32_t row_begin, int32_t row_end, int64_t cap, int32_t *cols,
                                          uint32_t *cnt, int16_t *cnt16);
/* Row-sum updates of the last window, one per delta row (same order as rows): exact int64 and the
 * reference's int view (RowSumAggregator.java:25-27; the reference drops an update whose int
 * value is 0, RowSumAggregator.java:66 -- the caller applies that filter on delta32). */
COOC_API int cooc_copy_window_rowsums(cooc_ctx *ctx, int32_t *items, int64_t *delta, int32_t *delta32);
/* Top-k of every rescored row: rows int32[n_topk], sizes int32[n_topk],
 * values int32[n_topk*topk], scores double[n_topk*topk] in IntDoublePriorityQueue heap order
 * (positions 1..size, least score first: IntDoublePriorityQueue.java:215-242). */
COOC_API int cooc_copy_window_topk(cooc_ctx *ctx, int32_t *rows, int32_t *sizes, int32_t *values, double *scores);

/* Global state snapshots. */
COOC_API int cooc_global_rowsums(cooc_ctx *ctx, int64_t *exact, int32_t *v32);          /* [n_items] each */
COOC_API int cooc_global_observed(cooc_ctx *ctx, int64_t *exact, int64_t *rescorer);   /* rescorer: sum of int deltas */
COOC_API int cooc_global_row_nnz(cooc_ctx *ctx, int32_t item, int64_t *nnz);
COOC_API int cooc_global_row(cooc_ctx *ctx, int32_t item, int32_t *cols, uint32_t *cnt, int16_t *cnt16);

/* ---- operator mirror: NonSampledUserInteractionCounterOneInputStreamOperator + aggregators ----
 * cooc_op_process_elements: Tuple3(user,item,ts) records in arrival order; records with
 * ts <= current watermark are dropped and counted (NonSampled...java:89-91).
 * cooc_op_process_watermark: advances the watermark and fires AT MOST ONE pending window with
 * maxTimestamp <= watermark (the earliest); sets *fired = 1 and fills *info if one fired (its
 * outputs are then readable with cooc_copy_window_*), *fired = 0 when nothing is due.  Callers
 * loop until *fired == 0, which mirrors the Flink timer service firing timers in timestamp order.
 * With a communicator of world > 1 the call is collective and a window is due when its maxTimestamp is at or
 * below the MINIMUM watermark over the ranks (agreed by an all-gather of the watermarks and of the earliest
 * pending windows); a rank whose watermark is ahead of that minimum waits inside the call until the other
 * ranks' watermarks catch up (every rank receives Long.MAX_VALUE at the end of a bounded input). */
COOC_API int cooc_op_process_elements(cooc_ctx *ctx, int64_t n, const int32_t *users, const int32_t *items,
                             const int64_t *ts, int64_t *n_late);
COOC_API int cooc_op_process_watermark(cooc_ctx *ctx, int64_t watermark, int32_t *fired, cooc_window_info *info);
/* counters[0] UserInteractionCounterLateElements, [1] UserInteractionCounterObservedCooccurrences,
 * [2] RowSumProcessWindowRowSum, [3] ItemRowRescorerRescoredItems, [4] rescorer observed. */
COOC_API int cooc_op_counters(cooc_ctx *ctx, int64_t *counters5);

/* ---- multi-GPU sharding layer (the keyBy(itemA) exchange, FlinkCooccurrences.java:152,163) ---------
 * Users are sharded over GPUs; each GPU's cooc_count_device result holds PARTIAL rows.  Row a is
 * owned by GPU (a mod n_parts).  The caller moves the packed partial rows with an all-to-all
 * (RCCL over xGMI, e.g. torch.distributed.all_to_all_single) and the row sums with an all-reduce.
 *   cooc_partition_plan   entries of the last cooc_count_device result per owner -> h_entries[n_parts]
 *   cooc_partition_pack   into caller DEVICE buffers, owner-major then ascending row:
 *                         d_row_nnz int32[n_items], d_entries uint64[sum h_entries] = (col << 32 | cnt)
 *   cooc_copy_rowsum_device  the last result's exact row sums into a caller device int64[n_items]
 *   cooc_merge_partitions for owner `part`: d_recv_row_nnz int32[n_parts * rows_owned] and
 *                         d_recv_entries (both source-major, as delivered by the all-to-all);
 *                         d_rowsum_global (the all-reduced row sums, may be NULL) checks every merged
 *                         row.  Result rows r = 0..n_rows-1 are items part + r * n_parts (borrowed
 *                         device views in *out; out->n_items = rows owned). */
COOC_API int cooc_partition_plan(cooc_ctx *ctx, int32_t n_parts, int64_t *h_entries);
COOC_API int cooc_partition_pack(cooc_ctx *ctx, int32_t n_parts, int32_t *d_row_nnz, uint64_t *d_entries,
                                 void *hip_stream);
COOC_API int cooc_copy_rowsum_device(cooc_ctx *ctx, int64_t *d_rowsum, void *hip_stream);
COOC_API int cooc_merge_partitions(cooc_ctx *ctx, int32_t n_parts, int32_t part, const int32_t *d_recv_row_nnz,
                                   const uint64_t *d_recv_entries, const int64_t *d_rowsum_global, void *hip_stream,
                                   cooc_device_result *out);

/* ---- communicator: the RCCL sharding layer behind the C-ABI ------------------------------------------
 * The reference's keyed exchanges -- keyBy(user) (FlinkCooccurrences.java:70), keyBy(ItemCooccurrences::
 * getItem) (:152) and rowSumStream.broadcast() (:163) -- as collectives inside the library, on the
 * context's caller stream, over RCCL (xGMI on one node).  One context per GPU process / Flink subtask; the
 * SURVEY §8(b) "refcounted device/RCCL singleton" is the process-wide RCCL library handle (dlopen'ed once;
 * a process that already loaded RCCL shares it).
 *   cooc_comm_unique_id  rank 0 creates the communicator id (COOC_COMM_ID_BYTES opaque bytes) and the
 *                        caller distributes it (Flink: the job graph's broadcast / a shared file; Python:
 *                        torch.distributed.broadcast).  Fails with COOC_ERR_HIP when RCCL is absent.
 *   cooc_comm_init       every rank: joins the world-size communicator as `rank` on the context's device.
 *   cooc_comm_init_ops   the same exchange over caller-provided collectives (any transport the caller has,
 *                        e.g. gloo in tests).  Each operation is collective over the ranks, takes device
 *                        pointers, returns 0 on success and must have completed with respect to hip_stream
 *                        when it returns (later work enqueued on that stream sees its result):
 *                          allreduce_sum_i64: d_buf[0, n) summed over the ranks, in place;
 *                          allgather: rank r's `bytes` at d_send land at d_recv + r * bytes;
 *                          alltoallv: send_bytes[p] bytes at d_send + send_off[p] go to rank p, which
 *                            receives them at d_recv + recv_off[sender]; recv_bytes[p] arrive from rank p
 *                            (host arrays of world entries). */
#define COOC_COMM_ID_BYTES 128
typedef struct cooc_comm_ops {
  int (*allreduce_sum_i64)(void *user, int64_t *d_buf, int64_t n, void *hip_stream);
  int (*allgather)(void *user, const void *d_send, void *d_recv, int64_t bytes, void *hip_stream);
  int (*alltoallv)(void *user, const void *d_send, const int64_t *send_off, const int64_t *send_bytes, void *d_recv,
                   const int64_t *recv_off, const int64_t *recv_bytes, void *hip_stream);
} cooc_comm_ops;
COOC_API int cooc_comm_unique_id(uint8_t *id);
COOC_API int cooc_comm_init(cooc_ctx *ctx, const uint8_t *id, int32_t rank, int32_t world);
COOC_API int cooc_comm_init_ops(cooc_ctx *ctx, int32_t rank, int32_t world, const cooc_comm_ops *ops, void *user);

/* One window of the multi-GPU large-universe job (n_items >= 40,320: C3 / C5), whole inside the library on
 * hip_stream: this rank's users (keyBy(user)) -> (1) local item frequencies, all-reduced (the planner's
 * column estimate and the owner map); (2) the row owner map: rows by descending global frequency (ties:
 * smaller id), the 4,096 most frequent placed greedily on the least loaded rank, the rest dealt in snake
 * order (cooc_snake_owner); (3) the histories all-gathered (one uneven all-to-all per array: every rank
 * sends its part to every peer at once, each pair over its own xGMI link); (4) the owned rows counted over
 * all users (cooc_count_device_owned: the keyBy(getItem) as ownership -- rows are complete on their owner,
 * nothing is merged); (5) the ordered pairs all-reduced.  *out: the owned rows (borrowed, as
 * cooc_count_device_owned); *info the totals and borrowed device views of the owner map and the global
 * item frequencies. */
typedef struct cooc_owned_info {
  int32_t part, n_parts;
  int64_t observed;           /* ordered pairs of the whole job (sum over the ranks) */
  int64_t local_observed;     /* ordered pairs of this rank's owned rows */
  int64_t n_users_all, n_interactions_all;
  int64_t gathered_bytes;     /* history bytes this rank received */
  const int32_t *owner;       /* device int32[n_items] */
  const int64_t *item_counts; /* device int64[n_items]: the all-reduced frequencies */
} cooc_owned_info;
COOC_API int cooc_count_owned(cooc_ctx *ctx, int64_t n_users, const int64_t *d_user_ptr, const int32_t *d_items,
                              int64_t n_interactions, void *hip_stream, cooc_owned_info *info,
                              cooc_device_result *out);
/* The same window from HOST arrays (a JVM subtask's buffered user shard: user_ptr int64[n_users+1] into
 * items), staged on the context's stream; *winfo as cooc_count_host (nnz, observed and rows with entries of
 * the OWNED rows).  The owned rows are then this context's batch result: cooc_copy_batch packs them (every
 * other row empty), cooc_topk_batch / cooc_topk_owned score them.  Replaces the p > 1 merge of partial
 * rows (ItemRowAggregator / RowSumAggregator windows keyed by item, FlinkCooccurrences.java:138-157) for a
 * one-window job. */
COOC_API int cooc_count_owned_host(cooc_ctx *ctx, int64_t n_users, const int64_t *user_ptr, const int32_t *items,
                                   cooc_owned_info *info, cooc_window_info *winfo);
/* C5 after cooc_count_owned: the owned rows' row sums all-reduced (the broadcast row-sum stream,
 * FlinkCooccurrences.java:163), then every owned row's LLR top-k against them (cooc_topk_batch_device).
 * d_rowsum_global (device int64[n_items], may be NULL) receives the all-reduced row sums. */
COOC_API int cooc_topk_owned(cooc_ctx *ctx, int32_t topk, int32_t flags, int32_t *d_sizes, int32_t *d_values,
                             double *d_scores, int64_t *d_rowsum_global, void *hip_stream);
/* cooc_topk_owned into the context's own buffers (a JVM subtask: GpuOwnedCooccurrenceTopKOperator), read back
 * with cooc_copy_topk_batch / cooc_copy_topk_batch_range / cooc_topk_items: every owned row's heap, scored
 * against the all-reduced row sums and the job's observed total.  Replaces the rescorer of
 * FlinkCooccurrences.java:162-167 (ItemRowRescorerTwoInputStreamOperator.java:195-226) for a one-window job. */
COOC_API int cooc_topk_owned_host(cooc_ctx *ctx, int32_t topk, int32_t flags);
/* Heaps of rows [row_begin, row_end) of the last cooc_topk_batch / cooc_topk_owned_host: sizes int32[n],
 * values int32[n*topk], scores double[n*topk] (n = row_end - row_begin, layout as cooc_copy_topk_batch).  topk
 * is the caller's buffer width and must equal the topk of that call: anything else is COOC_ERR_ARG and nothing
 * is written (the buffers are sized from it). */
COOC_API int cooc_copy_topk_batch_range(cooc_ctx *ctx, int32_t row_begin, int32_t row_end, int32_t topk,
                                        int32_t *sizes, int32_t *values, double *scores);
/* Every rank's `value` (collective over the communicator): out int64[world] in rank order.  The JVM operators
 * agree on the window they fire with it (a subtask with no records of its own joins the same window). */
COOC_API int cooc_comm_allgather_i64(cooc_ctx *ctx, int64_t value, int64_t *out);
/* The owner map of step (2) on the host (no device): counts int64[n_items] -> owner int32[n_items]. */
COOC_API int cooc_snake_owner(const int64_t *counts, int32_t n_items, int32_t world, int32_t head, int32_t *owner);

/* ---- sharded records (multi-GPU: the keyBy(itemA) of FlinkCooccurrences.java:152 on pair RECORDS) -
 * Users are sharded over n_parts GPUs (keyBy(user), :70); row a is owned by part a mod n_parts.  The
 * reference ships each pair record (itemA, the user's history) to the owner of itemA; here every
 * part ships its users' histories once (the caller all-gathers the u16 arenas) and one 8-B
 * descriptor per record (the caller all-to-alls them by owner), and each owner reduces complete
 * rows: no partial counts are exchanged and nothing is merged.
 *   cooc_shard_plan   this part's users -> into caller DEVICE buffers: d_desc uint64[n_interactions]
 *                     (descriptors grouped by owner, then by owned row), d_row_counts int32[n_items]
 *                     (row counts in the same owner-major order: owner o's rows_owned(o) counts are
 *                     contiguous), d_arena uint16[arena_cap >= n_interactions + 7 n_users + 16];
 *                     h_send[n_parts] = descriptors per owner, h_info[0] = arena ids used (a multiple
 *                     of 8), h_info[1] = this part's ordered pairs.
 *   cooc_shard_count  owner `part`: d_recv_row_counts int32[n_parts * rows_owned] and d_recv_desc
 *                     (source-major, as delivered by the all-to-all), d_arena_all the all-gathered
 *                     arenas with source s at s * arena_stride ids.  Result rows r = 0..n_rows-1 are
 *                     items part + r * n_parts (borrowed device views in *out; out->n_items = rows
 *                     owned), complete: counts, row sums and the overflow check are final. */
COOC_API int cooc_shard_plan(cooc_ctx *ctx, int64_t n_users, const int64_t *d_user_ptr, const int32_t *d_items,
                             int64_t n_interactions, int32_t n_parts, uint64_t *d_desc, int32_t *d_row_counts,
                             uint16_t *d_arena, int64_t arena_cap, void *hip_stream, int64_t *h_send,
                             int64_t *h_info);
COOC_API int cooc_shard_count(cooc_ctx *ctx, int32_t n_parts, int32_t part, const int32_t *d_recv_row_counts,
                              const uint64_t *d_recv_desc, int64_t n_recv, const uint16_t *d_arena_all,
                              int64_t arena_stride, void *hip_stream, cooc_device_result *out);

/* ---- ItemCooccurrences wire codec (ItemCooccurrences.java:113-147, Kryo 2.24 primitives) --------
 * Host-only (no device calls, no context).  A record is (item, increment int16, size other items):
 * varint item, big-endian int16 increment, varint size', size' varints -- every varint is Kryo's
 * writeInt(v, true).  For a mixed deployment that keeps the Java emitter or the Java reducer.
 *   cooc_records_encode  n records: items int32[n], increments int16[n], ks int32[n] (slot k is
 *                        skipped, ItemCooccurrences.java:124-131; NULL = all -1), rec_ptr
 *                        int64[n+1] into others.  out == NULL: *n_bytes = encoded size only;
 *                        else out must hold out_cap >= *n_bytes bytes.
 *   cooc_records_decode  bytes -> *n_records, *n_others; pass NULL arrays to size them, then
 *                        items int32[n_records], increments int16[n_records], rec_ptr
 *                        int64[n_records+1], others int32[n_others] (any may be NULL).  A truncated
 *                        record or a negative size fails with COOC_ERR_ARG. */
COOC_API int cooc_records_encode(int64_t n_records, const int32_t *items, const int16_t *increments, const int32_t *ks,
                                 const int64_t *rec_ptr, const int32_t *others, uint8_t *out, int64_t out_cap,
                                 int64_t *n_bytes);
COOC_API int cooc_records_decode(const uint8_t *bytes, int64_t n_bytes, int64_t *n_records, int64_t *n_others,
                                 int32_t *items, int16_t *increments, int64_t *rec_ptr, int32_t *others);

/* ---- text ingest (FlinkCooccurrences.java:55-61,207-229: TextInputFormat + InteractionLineSplitter) --
 * Host-only.  text: n_bytes of '\n'-delimited "user,item,timestamp" lines ("\r\n" accepted, fields after
 * the third ignored, as String.split(",") + Integer.valueOf / Long.valueOf).  users == NULL (or
 * items / ts NULL): *n_records = the number of lines only.  Else parses up to cap records; a line
 * that the reference's splitter rejects (NumberFormatException / ArrayIndexOutOfBoundsException)
 * fails with COOC_ERR_ARG and its 0-based index in *bad_line.  The watermark of the reference's
 * AscendingTimestampExtractor after a prefix of records is (largest timestamp so far) - 1. */
COOC_API int cooc_parse_interactions(const char *text, int64_t n_bytes, int64_t cap, int32_t *users, int32_t *items,
                                     int64_t *ts, int64_t *n_records, int64_t *bad_line);

/* ---- invariant checks of a batch result (the reference's DEVELOPMENT_MODE checks) ---------------
 * FlinkCooccurrences.java:34 switches on, among others, the row-sum consistency check of the rescorer
 * (ItemRowRescorer...java:183-193: the sum of a row == the item's row sum).  cooc_verify_batch runs it,
 * and the checks of this library's CSR contract, over the whole last cooc_count_device /
 * cooc_count_device_owned result on hip_stream (then synchronises it).  out8 (host int64[8]):
 *   [0] sum of all counts         [1] sum of the row sums (== [0] == observed for a whole result)
 *   [2] entries                   [3] rows whose counts do not sum to their row sum
 *   [4] rows with a bad entry: columns not strictly ascending or outside [0, n_items), a count of 0
 *       (dense layout: row_nnz[a] != the row's non-zero cells)
 *   [5] entries with C[a,b] != C[b,a] (only with COOC_VERIFY_SYMMETRY, padded CSR of a whole result;
 *       else -1)                  [6], [7] 0
 * d_row_checksum (device uint64[n_items], may be NULL): per row, the sum over its keys of
 * splitmix64((col << 32) ^ count) mod 2^64 (splitmix64(x): x += 0x9E3779B97F4A7C15;
 * x = (x ^ x >> 30) * 0xBF58476D1CE4E5B9; x = (x ^ x >> 27) * 0x94D049BB133111EB; x ^ x >> 31), a
 * fingerprint to compare the result row by row with an independent restatement without copying it
 * out. */
#define COOC_VERIFY_SYMMETRY 1
COOC_API int cooc_verify_batch(cooc_ctx *ctx, int32_t flags, uint64_t *d_row_checksum, int64_t *out8,
                               void *hip_stream);

/* ---- diagnostics (not part of the reference surface) ------------------------------------------
 * Kernel timing of the dominant kernel (the accumulate kernel) with HIP events recorded on the
 * stream it is launched on; read back after a call that ran it. */
COOC_API int cooc_set_kernel_timing(cooc_ctx *ctx, int32_t enable);
COOC_API int cooc_last_kernel_ms(cooc_ctx *ctx, float *accumulate_ms);
/* Rows (and their ordered pairs) that the last large-universe count sent through the sort +
 * segmented-reduce path (hash table overflow, or COOC_FLAG_SORT_ROWS). */
COOC_API int cooc_last_sort_rows(cooc_ctx *ctx, int64_t *rows, int64_t *pairs);
/* Self-test of the planner's single-pass device prefix sum (no context): d_out[i] = d_in[0] + .. + d_in[i]
 * (flags & 1) or + .. + d_in[i-1] over device arrays of n elements, on hip_stream (then synchronised).
 * flags: 1 inclusive, 2 tiles staged through LDS (else vectorised loads), 4 int32 output (else int64), 8 int32
 * input (else int64).  *diag (may be NULL) gets the scan's diagnostic word (bit 16: a look-back stopped waiting
 * and summed its prefix from the input). */
COOC_API int cooc_selftest_scan(const void *d_in, void *d_out, int64_t n, int32_t flags, int64_t *diag,
                                void *hip_stream);
/* Self-test of the planner's radix sort (no context): (d_keys_out, d_vals_out)[0, n) = (d_keys_in, d_vals_in)
 * stably sorted by key bits [bit0, bit1) (descending != 0: by the complemented bits, equal keys in input order),
 * keys of key_bytes (4 or 8) bytes, 32-bit values; device arrays, on hip_stream (then synchronised). */
COOC_API int cooc_selftest_radix(const void *d_keys_in, const void *d_vals_in, void *d_keys_out, void *d_vals_out,
                                 int64_t n, int32_t key_bytes, int32_t bit0, int32_t bit1, int32_t descending,
                                 void *hip_stream);
/* Self-test of the planner's flag compaction: d_out[0, *d_n_sel) = the indices i < n with d_flags[i] != 0,
 * ascending (device arrays; *d_n_sel is a device int32). */
COOC_API int cooc_selftest_select(const uint8_t *d_flags, int64_t n, int32_t *d_out, int32_t *d_n_sel,
                                  void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* COOC_H_ */
