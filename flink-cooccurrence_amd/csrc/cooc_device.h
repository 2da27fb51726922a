// cooc_device.h — internal C++ interface between the C-ABI (cooc_capi.cpp) and the HIP kernels.
//
// The device pipeline reduces "contributions" into per-row dense LDS accumulators.  A
// contribution is (row a, segment of one user's history in the device arena): the reference's
// NonSampled...java:113-165 expansion of one window is exactly
//   for every user u expanded in the window, with resident history length `old` and `len` items
//   after appending the window's items (old + new, arrival order):
//     position p >= old (a NEW interaction x_p):  row x_p += the whole list  [0, len), then -1 at x_p
//     position p <  old (an OLD interaction x_p): row x_p += the new part     [old, len)
// which covers every ordered position pair (p != q) whose later position is new — the pairs the
// reference emits in that window (ITEM records (x, h, +1) and (o, x, +1), :138-151).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <string>

namespace cooc {

struct Status {
  int code = 0;  // cooc_status
  std::string msg;
  bool ok() const { return code == 0; }
  static Status Ok() { return {}; }
};

#define COOC_HIP_TRY(expr)                                                                      \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess)                                                                       \
      return ::cooc::Status{3, std::string(#expr) + ": " + hipGetErrorString(e_)};              \
  } while (0)

#define COOC_TRY(expr)            \
  do {                            \
    ::cooc::Status s_ = (expr);   \
    if (!s_.ok()) return s_;      \
  } while (0)

// int32 -> int64 widening for prefix sums whose totals may exceed 2^31 (hipCUB accumulates in the
// input value type).
struct WidenI64 {
  __host__ __device__ int64_t operator()(int32_t v) const { return int64_t(v); }
};

// Grow-only device buffer (the workspace of one context).  Never shrinks, so steady-state
// windows perform no hipMalloc.
struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  Status reserve(size_t bytes);
  void release();
  template <class T>
  T *as() const { return static_cast<T *>(p); }
};

// The users expanded in one window, all device pointers.
struct ActiveUsers {
  int64_t n_active = 0;
  const int64_t *off = nullptr;    // [n_active] arena offset of the user's history
  const int32_t *len = nullptr;    // [n_active] history length after the window (old + new)
  const int32_t *old = nullptr;    // [n_active] history length before the window
  const int64_t *cbase = nullptr;  // [n_active + 1] exclusive prefix of len (contribution slots)
  int64_t n_contrib = 0;           // == cbase[n_active] (host copy)
  int64_t n_new = 0;               // interactions of the window == sum(len - old) (host copy)
  const int32_t *arena = nullptr;  // item ids of all histories
  const uint16_t *arena16 = nullptr;  // optional u16 mirror of arena (n_items <= 40,704); else narrowed per run
  int64_t arena_span = 0;             // arena entries [0, span) the contributions may reference
};

// One row's share of the work (heavy rows are split over several chunks).
struct Chunk {
  int32_t row;
  int32_t split;  // staging slot of a split row, -1 when the row is one chunk
  int64_t begin;  // contribution range [begin, end) in row-sorted order
  int64_t end;
  int64_t pad;
};

// Scalars of one run (device-side, copied to a pinned host mirror once per run).
struct PlanTotals {
  int64_t n_chunks;
  int64_t cap_total;  // padded output entries
  int64_t n_split;
  int64_t work_total; // sum over contributions of segment length (ordered pairs + self terms)
  int64_t nnz_total;  // filled after the run
  int64_t err;        // bit 0: item id out of range, bit 1: uint32 count overflow
  // batch planner (run_batch) statistics of the user histories
  int64_t sum_l2;     // sum_u n_u^2  (= ordered pairs + self terms)
  int64_t sum_lpl;    // sum_u n_u * pad8(n_u): padded partner ids read
  int64_t max_len;    // longest history
  int64_t n_long;     // histories longer than kFillThread (filled by a workgroup each)
  // large-universe path (run_sparse)
  int64_t est_nnz;       // expected distinct keys (planner estimate, sizes the output region)
  int64_t n_split_work;  // work items of the split rows
  int64_t n_active;      // rows with at least one contribution
  int64_t max_tail;      // largest expected gather tail (pairs outside tile 0) of a work item
  int64_t n_gather_rows;  // whole rows in gather mode (their work items get bucket-start slots)
  int64_t n_gather;       // bucket-start slots handed out by the queue builder
  int64_t bad_row;        // a row whose counts failed the row-sum check (err bit 1), for the message
  int64_t self_total;     // contributions whose walk includes their own position (pairs p == p removed)
  int64_t n_deferred;     // whole rows handed to the sort + segmented-reduce path (hash table overflow)
  int64_t n_tiny;         // whole rows of <= kTinyW pairs (the queue's tail): one wave each (k_sp_tiny)
  int64_t tiny_ctr;       // k_sp_tiny's work counter
  int64_t n_small;        // whole rows of kTinyW < W <= kSmallW pairs (before the tiny ones): a workgroup each (k_sp_small)
  int64_t small_ctr;      // k_sp_small's work counter
  int64_t srb_ctr;        // k_srb_row's row counter (the deferred rows)
  int64_t ts_pairs;       // pairs of the tiny and small rows (sorted by k_sp_tiny / k_sp_small)
  int64_t n_mid;          // whole rows of at most kMidW pairs above the small ones: k_sp_main's mid shape
  int64_t max_tail_mid;   // largest expected gather tail of a mid row (sizes the mid launch's scratch)
};

// One streaming window through the large-universe path in one pass (NonSampled...java:129-161): the CSR
// handed to run_sparse holds 2 lists per user, A_j = the history after the window and B_j = the window's
// new items; a new position of A_j walks A_j, an old one walks B_j (k_sp_window_contribs).  All device
// pointers; n_contrib = sum of the |A_j| = cbase[n_users] (host copy).
struct SparseWindow {
  int64_t n_users = 0;
  const int32_t *old = nullptr;    // [n_users] history length before the window
  const int64_t *cbase = nullptr;  // [n_users + 1] exclusive prefix of |A_j|
  int64_t n_contrib = 0;
};

// Result of a run: padded CSR over all M rows, device pointers owned by the Counter.
struct CountResult {
  int64_t *row_base = nullptr;
  int32_t *row_nnz = nullptr;
  int32_t *col = nullptr;
  uint32_t *cnt = nullptr;
  int64_t *rowsum = nullptr;
  uint32_t *dense = nullptr;  // dense output: row-major [M x M] counts (row_base / col / cnt unused)
  // the column order of the rows: ascending rank_of[col] (the large-universe batch path puts the batch's
  // 16,384 most frequent items first, then the rest, each group by id); NULL = ascending column id
  const int32_t *rank_of = nullptr;
  bool unordered = false;  // COOC_FLAG_ANY_ORDER: the rows' entries in no particular order
  int64_t nnz = 0;
  int64_t observed = 0;  // ordered pairs of the run
  int64_t work = 0;
};

// Kernel timing hooks for the benchmark (HIP events recorded on the run's stream).
struct KernelTimer {
  hipEvent_t acc_begin = nullptr, acc_end = nullptr;
  bool enabled = false;
};

class Counter {
 public:
  Status init(int32_t n_items);
  void release();
  ~Counter() { release(); }

  // One window over empty histories straight from a device CSR (user_ptr int64[U+1], items
  // int32[N]): the batch planner (per-block item histograms -> transpose of A by counting sort) and
  // k_acc_batch.  Needs n_items < kBatchMaxItems (one LDS row + pad sink + descriptors); returns the same padded
  // CSR as run().  Synchronises `stream` once (to size chunks and the output region).
  Status run_batch(int64_t n_users, const int64_t *user_ptr, const int32_t *items, int64_t n, hipStream_t stream,
                   CountResult *out, KernelTimer *timer = nullptr);
  bool batch_ok() const { return M_ < kBatchMaxItems && !general_only_; }
  // the large-universe planner: n_items >= kBatchMaxItems, or any n_items with COOC_FLAG_GENERAL_PLANNER
  // n_items >= kBatchMaxItems: one window over empty histories through the large-universe path
  // (cooc_sparse.hip: per-row workgroups, LDS hash / dense-tile chunks, split staging rows).  Same
  // padded CSR result as run().  Synchronises `stream` twice (plan totals, output-region check).
  // owner != NULL (multi-GPU): only the rows a with owner[a] == part are counted (over every user
  // given), and the planner's column frequencies come from freq (int64[n_items], n_freq in total:
  // the global log's item counts); other rows come out empty.
  Status run_sparse(int64_t n_users, const int64_t *user_ptr, const int32_t *items, int64_t n, hipStream_t stream,
                    CountResult *out, KernelTimer *timer = nullptr, const int32_t *owner = nullptr,
                    int32_t part = 0, const int64_t *freq = nullptr, int64_t n_freq = 0,
                    const SparseWindow *win = nullptr);
  bool sparse() const { return M_ >= kBatchMaxItems || general_only_; }
  // A streaming window (resident histories) through the batch planner and k_acc_batch; needs
  // batch_ok().  Same padded CSR result as run().  Synchronises `stream` once.
  Status run_window(const ActiveUsers &au, hipStream_t stream, CountResult *out, KernelTimer *timer = nullptr);
  // COOC_FLAG_GENERAL_PLANNER: every window through the large-universe planner (run_sparse).
  void set_general_only(bool g) { general_only_ = g; }

  // Sharded records (W parts, owner(a) = a mod W).  shard_plan: this part's users -> its padded
  // u16 arena (arena[arena_cap >= n + 7 U + 16]), descriptors grouped by owner (desc[n]) and row
  // counts in owner-major order (row_counts[n_items]); h_send[W] descriptors per owner, the arena's
  // ids and this part's ordered pairs.  Synchronises `stream`.
  Status shard_plan(int64_t n_users, const int64_t *user_ptr, const int32_t *items, int64_t n, int32_t W,
                    hipStream_t stream, uint64_t *desc, int32_t *row_counts, uint16_t *arena, int64_t arena_cap,
                    int64_t *h_send, int64_t *h_arena_ids, int64_t *h_observed);
  // shard_count: the owned rows (part + r W) from every source's row counts [W x R] and descriptor
  // segments (source order) over the all-gathered arenas (source s at s * arena_stride ids).
  Status shard_count(int32_t W, int32_t part, const int32_t *recv_counts, const uint64_t *recv_desc, int64_t n_recv,
                     const uint16_t *arena_all, int64_t arena_stride, hipStream_t stream, CountResult *out,
                     KernelTimer *timer = nullptr);
  int32_t last_rows() const { return last_rows_; }
  // COOC_FLAG_SORT_ROWS: every whole row of the large-universe path through the sort + segmented-reduce
  // path (otherwise only rows whose LDS hash table overflowed); rows and pairs it took in the last run
  void set_sort_rows(bool on) { sort_rows_ = on; }
  void set_relabel(bool on) { relabel_ = on; }
  void set_any_order(bool on) { any_order_ = on; }
  const int32_t *last_rank_of() const { return last_pos_of_; }
  int64_t last_deferred_rows() const { return last_deferred_; }
  int64_t last_deferred_pairs() const { return last_deferred_pairs_; }
  static constexpr int32_t kBatchMaxItems = 40320;

  // Output layout of run_batch: 0 = auto (dense when P >= M^2 / 2), 1 = sparse CSR, 2 = dense.
  void set_output_layout(int pref) { output_pref_ = pref; }
  bool last_dense() const { return dense_mode_; }
  const uint32_t *last_dense_counts() const { return dense_mode_ ? dense_.as<uint32_t>() : nullptr; }

  // Pack the result of the last run into contiguous CSR (device), for copy-out.
  Status pack(hipStream_t stream, int64_t **row_ptr, int32_t **col, uint32_t **cnt);
  // Copy the device totals of the last run (the stream must have drained).
  Status read_totals(PlanTotals *t);
  const int64_t *last_rowsum() const { return rowsum_.as<int64_t>(); }
  const int32_t *last_row_nnz() const { return row_nnz_.as<int32_t>(); }
  const int64_t *last_row_base() const { return row_base_.as<int64_t>(); }
  const int32_t *last_col() const { return col_.as<int32_t>(); }
  const uint32_t *last_cnt() const { return cnt_.as<uint32_t>(); }
  int32_t n_items() const { return M_; }

 private:
  Status plan_local(int64_t U, const int64_t *up, const int32_t *items, int64_t n, int32_t W, hipStream_t s,
                    uint64_t *desc, uint16_t *arena, int64_t arena_cap, const int32_t *old = nullptr,
                    const int64_t *hoff = nullptr);
  Status accumulate_rows(int32_t R, int32_t W, int32_t part, const int64_t *row_ptr, const int32_t *rcnt,
                         const uint64_t *desc, const uint16_t *arena, int64_t n, int64_t n_self, bool sparse_only,
                         hipStream_t s, CountResult *out, KernelTimer *timer);

  int32_t M_ = 0;
  int n_cu_ = 256;
  // workspace
  DevBuf keys_in_, vals_in_, keys_out_, vals_out_, sort_tmp_, epre_;
  DevBuf row_ptr_, row_work_, row_nch_, row_cap_, row_split_, order_keys_, order_;
  DevBuf ord_nch_, ord_cbase_, row_base_, split_slot_, split_row_, chunks_, tot_, queue_;
  DevBuf col_, cnt_, staging_, row_nnz_, rowsum_;
  DevBuf pk_row_ptr_, pk_col_, pk_cnt_, split_sum_, tarena_;
  int64_t bump_cap_ = 0;    // k_acc_batch sparse output: entries in the bump region
  DevBuf bump_, seg_off_;  // seg_off_: sharded records, per (source, owned row) segment offsets
  DevBuf plen_, poff_;
  DevBuf bh_, uidx_, long_, rcnt_, desc_;  // batch planner: block histograms, user of each interaction,
                                           // long lists, row counts, descriptors
  int output_pref_ = 0;               // set_output_layout
  bool dense_mode_ = false;           // the last run's output is dense_
  DevBuf dense_, send_, witems_;
  // large-universe path: tile-grouped arena, tile starts, per-row work and plan, estimates, queue
  DevBuf sp_arena_, sp_tb_, sp_roww_, sp_pstart_, sp_pdense_, sp_est_, sp_queue_, sp_ownc_, sp_ownoff_, sp_pbase_, sp_scr_, sp_hz_;
  DevBuf sp_spre_;  // streaming windows: prefix of the contributions' self flags
  DevBuf sp_ulen_;     // the lists' lengths (u32) for the pair-work prefix
  DevBuf scan_state_;  // the planner prefix sums' tile statuses (cooc_scan.h)
  DevBuf sp_arena0_;  // the lists' tile-0 ids as u16 (arena0; sp_arena_ holds the rest)
  // sort + segmented-reduce path of deferred rows: the deferred list, keys (x2), runs, per-batch tables
  DevBuf sp_defer_, sr_keys_, sr_ukeys_, sr_ucnt_, sr_aux_;
  int64_t last_deferred_ = 0, last_deferred_pairs_ = 0;
  int32_t last_hot_overlap_ = -1;  // hot items with an id below kTW at the last relabel decision (-1: none)
  bool sort_rows_ = false;  // COOC_FLAG_SORT_ROWS
  // batch windows of the large-universe path: the kTW most frequent items renumbered into tile 0 (ascending
  // ids), the others at id + kTW; skipped when 15/16 of them have ids < kTW (off: COOC_FLAG_COLUMN_ORDER); the
  // last run's maps (NULL without a relabel)
  bool relabel_ = true;
  bool any_order_ = false;  // COOC_FLAG_ANY_ORDER: hash chunks emitted in slot order (batch results)
  DevBuf sp_rank_, sp_rkeys_, sp_bits_;  // (sp_bits_: the hot-column and owned-row bitmaps of the user passes)
  const int32_t *last_hot_col_ = nullptr, *last_pos_of_ = nullptr;
  int32_t last_mc_ = 0;       // columns of the last run's (relabelled) space
  // deferred rows through the library radix sort (COOC_SR_HIPCUB=1, A/B) instead of k_srb_row
  bool srb_hipcub_ = getenv("COOC_SR_HIPCUB") && getenv("COOC_SR_HIPCUB")[0] == '1';
  bool small_off_ = getenv("COOC_SP_SMALL") && getenv("COOC_SP_SMALL")[0] == '0';  // (A/B: small rows in k_sp_main)
  bool mid_off_ = getenv("COOC_SP_MID") && getenv("COOC_SP_MID")[0] == '0';  // (A/B: mid rows in the big shape)
  // the mid-row and small-row launches on streams of their own, forked from and joined back to the caller's
  // stream, so that their workgroups fill the CUs the big launch's last workgroups leave idle (COOC_SP_FORK=0:
  // one after the other on the caller's stream)
  int fork_mode_ = getenv("COOC_SP_FORK") ? atoi(getenv("COOC_SP_FORK")) : 0;  // (A/B: 1 fork at the start, 2 small rows beside the mid launch)
  hipStream_t aux_[2] = {nullptr, nullptr};
  hipEvent_t ev_fork_ = nullptr, ev_join_[2] = {nullptr, nullptr};
  DevBuf sp_scr_mid_;      // the mid launch's gather scratch
  int64_t last_mid_grid_ = 0;
  Status run_deferred(int64_t n_def, int32_t T, const int64_t *row_ptr, const int64_t *epre, const uint32_t *vals,
                      const int64_t *spre, int64_t cap, hipStream_t s);
  bool general_only_ = false;
  int32_t last_rows_ = 0;             // rows of the last batch result (n_items, or the owned rows)
  static constexpr int64_t chunk_work_ = int64_t(1) << 22;  // pairs per chunk of the batch planner
  PlanTotals *h_tot_ = nullptr;  // pinned
};

// Item frequencies of a device item array into counts int64[M] (zeroed first); ids outside [0, M) are
// not counted.
Status launch_item_counts(hipStream_t s, const int32_t *items, int64_t n, int32_t M, int64_t *counts);

// Invariant checks + per-row fingerprints of a batch result (cooc_verify.hip): d_tot uint64[8] =
// {sum of counts, sum of row sums, entries, rows whose counts miss their row sum, rows with a bad
// entry, asymmetric entries (symmetry only), 0, 0}; d_cs (may be NULL) uint64[M] row checksums.
Status launch_verify(hipStream_t s, int32_t M, const CountResult &r, bool symmetry, uint64_t *d_cs,
                     unsigned long long *d_tot);

// Sparse global rows of the streaming state (n_items >= 40,320; the rescorer's itemRows,
// ItemRowRescorer...java:35,171-177): row a = len[a] (column, count) entries in ascending column order
// at base[a] of the arena (col, cnt); kernels in cooc_stream.hip.
struct GlobalSparse {
  DevBuf base, len, col, cnt, flag, newpre, nbase, bump_dev, opos, chunk_pre;
  int64_t cap = 0, bump = 0, live = 0;
  void release() {
    DevBuf *all[] = {&base, &len, &col, &cnt, &flag, &newpre, &nbase, &bump_dev, &opos, &chunk_pre};
    for (DevBuf *b : all) b->release();
    cap = bump = live = 0;
  }
};

}  // namespace cooc
