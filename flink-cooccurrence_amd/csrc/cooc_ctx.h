// cooc_ctx.h — the context behind the C-ABI handle: one per Flink subtask.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/cooc.h"
#include "cooc_comm.h"
#include "cooc_device.h"
#include "cooc_shard.h"

struct cooc_ctx;

namespace cooc {

// Resident streaming state: per-user histories (device arena), global rows (dense uint32
// [n_items x n_items] in HBM), global row sums, the rescorer's observed total, and the outputs of
// the last finished window.  Restates NonSampled...java:129-161 (history), ItemRowRescorer...java:
// 33-41,144-241 (global state, merge, rescoring).
class StreamState {
 public:
  Status submit(cooc_ctx &ctx, int64_t ts, int32_t n_users, const int32_t *user_ids, const int64_t *user_ptr,
                const int32_t *items);
  Status finish(cooc_ctx &ctx, int64_t ts, cooc_window_info *info);
  Status copy_delta(cooc_ctx &ctx, int32_t *rows, int64_t *row_ptr, int32_t *cols, uint32_t *cnt, int16_t *cnt16);
  // entries of the delta rows [r0, r1) (row indices as in copy_delta): a window streams out in row ranges
  Status copy_delta_range(cooc_ctx &ctx, int32_t r0, int32_t r1, int64_t cap, int32_t *cols, uint32_t *cnt,
                          int16_t *cnt16);
  Status copy_rowsums(cooc_ctx &ctx, int32_t *items, int64_t *delta, int32_t *delta32);
  Status copy_topk(cooc_ctx &ctx, int32_t *rows, int32_t *sizes, int32_t *values, double *scores);
  Status global_rowsums(cooc_ctx &ctx, int64_t *exact, int32_t *v32);
  Status global_row_nnz(cooc_ctx &ctx, int32_t item, int64_t *nnz);
  Status global_row(cooc_ctx &ctx, int32_t item, int32_t *cols, uint32_t *cnt, int16_t *cnt16);
  void release();

  int64_t observed_exact = 0;  // UserInteractionCounterObservedCooccurrences (NonSampled...java:80,153)
  int64_t observed_ref = 0;    // ItemRowRescorer observedCooccurrences: long += int delta (:37,154)
  int64_t rowsum_acc = 0;      // RowSumProcessWindowRowSum (RowSumAggregator.java:50,67)
  int64_t rescored_items = 0;  // ItemRowRescorerRescoredItems (ItemRowRescorer...java:60,169)

 private:
  Status ensure_global(cooc_ctx &ctx);
  int32_t slot_for(int32_t user_id);
  Status pack_delta(cooc_ctx &ctx);
  Status copy_entries(int64_t e0, int64_t e1, int32_t *cols, uint32_t *cnt, int16_t *cnt16);
  Status grow_arena(cooc_ctx &ctx, int64_t need);
  // p > 1 subtasks (a communicator on the context): the window's partial delta rows routed to their owners
  // (a mod world) and merged there, the row-sum deltas and the observed pairs all-reduced
  Status exchange_window(cooc_ctx &ctx, hipStream_t s, const CountResult *r, int64_t obs_local, int64_t *obs_total);
  Status finish_owned(cooc_ctx &ctx, hipStream_t s, int64_t ts, int64_t obs_local, int64_t obs_total,
                      cooc_window_info *info);
  // n_items >= 40,320: one window through the large-universe planner, old / new positions in one pass
  Status count_large_window(cooc_ctx &ctx, hipStream_t s, int64_t n_act, const std::vector<int64_t> &act_off,
                            const std::vector<int32_t> &act_len, const std::vector<int32_t> &act_old,
                            int64_t n_full, CountResult *r);

  // host metadata of the per-user histories
  std::unordered_map<int32_t, int32_t> slot_of_;  // user ids outside [0, 2^26)
  std::vector<int32_t> dense_slot_;               // user ids in [0, 2^26)
  std::vector<int64_t> h_off_;
  std::vector<int32_t> h_len_, h_cap_;
  int64_t arena_used_ = 0;
  DevBuf arena_;
  // staged window
  bool staged_ = false;
  int64_t staged_ts_ = 0;
  int64_t window_seq_ = 0;
  int32_t n_staged_ = 0;
  std::vector<int64_t> staged_stamp_;  // per slot: window_seq_ when staged in the current window
  std::vector<int32_t> staged_pos_;    // per slot: index into staged_slots_/staged_items_
  std::vector<int32_t> staged_slots_;
  std::vector<std::vector<int32_t>> staged_items_;  // reused across windows
  // device uploads of one window
  DevBuf d_act_off_, d_act_len_, d_act_old_, d_cbase_, d_new_items_, d_new_dst_ptr_, d_new_dst_, d_reloc_;
  // large-universe windows: the users' whole histories and new items side by side (2 lists per user)
  DevBuf d_lw_items_, d_lw_up2_, d_lw_dsta_, d_lw_dstb_, d_lw_srcb_, d_lw_lenb_;
  // global state
  bool global_ready_ = false;
  bool sparse_global_ = false;  // n_items >= 40,320: sorted row slabs (gs_) instead of the dense matrix
  GlobalSparse gs_;
  DevBuf d_global_, d_grs_, d_touched_, d_scan_tmp_, d_scal_, d_topk_val_, d_topk_score_, d_topk_size_, d_llr_terms_;
  // last window
  bool have_window_ = false;
  bool empty_window_ = false;  // the last window had no interaction left after user_cut
  cooc_window_info last_{};
  int32_t n_touched_ = 0;
  // the last window's delta rows packed for copy-out (once per window)
  bool delta_packed_ = false;
  int64_t *pk_rp_ = nullptr;
  int32_t *pk_col_ = nullptr;
  uint32_t *pk_cnt_ = nullptr;
  std::vector<int32_t> delta_rows_;
  std::vector<int64_t> delta_start_;
  // p > 1: the last window's owned delta rows (an M-row view over the merge's rows), the all-reduced window row
  // sums, the exchange buffers, and the packed copy-out of the owned rows
  bool owned_window_ = false;
  const int32_t *own_col_ = nullptr;
  const uint32_t *own_cnt_ = nullptr;
  DevBuf d_own_base_, d_own_nnz_, d_rs_win_, d_x_nnz_, d_x_ent_, d_r_nnz_, d_r_ent_, d_x_h_, d_zero_;
  DevBuf d_own_rp_, d_own_pcol_, d_own_pcnt_;
};

// NonSampledUserInteractionCounterOneInputStreamOperator mirror: late-element drop, tumbling
// window assignment, per-window buffering in arrival order, watermark-driven firing
// (NonSampled...java:84-165).
class Operator {
 public:
  Status process_elements(cooc_ctx &ctx, int64_t n, const int32_t *users, const int32_t *items, const int64_t *ts,
                          int64_t *n_late);
  Status process_watermark(cooc_ctx &ctx, int64_t watermark, int32_t *fired, cooc_window_info *info);

  int64_t watermark = INT64_MIN;  // timerService.currentWatermark() (this subtask's own)
  int64_t late_elements = 0;      // UserInteractionCounterLateElements

 private:
  struct Pending {
    std::vector<int32_t> users, items;
  };
  Status fire(cooc_ctx &ctx, int64_t max_ts, bool mine, int32_t *fired, cooc_window_info *info);
  std::map<int64_t, Pending> pending_;  // window.maxTimestamp() -> buffered interactions
  // p > 1: the watermark every subtask has passed (the minimum of their watermarks at the last agreement
  // step; identical on every subtask), and whether the last step fired a window (then the next call runs
  // another step whatever its watermark, so that every subtask runs the same sequence of collectives)
  int64_t agreed_ = INT64_MIN;
  bool regather_ = false;
};

}  // namespace cooc

struct cooc_ctx {
  cooc::Status init(const cooc_config &cfg);
  ~cooc_ctx();

  cooc::Status count_device(int64_t n_users, const int64_t *d_user_ptr, const int32_t *d_items, int64_t n_interactions,
                            hipStream_t s, cooc_device_result *out);
  cooc::Status count_device_owned(int64_t n_users, const int64_t *d_user_ptr, const int32_t *d_items,
                                  int64_t n_interactions, const int32_t *d_owner, int32_t part,
                                  const int64_t *d_item_counts, int64_t n_total, hipStream_t s,
                                  cooc_device_result *out);
  // user_cut > 0: replaces the CSR by its capped copy (b_cut_*); no-op otherwise
  cooc::Status apply_user_cut(int64_t n_users, const int64_t **d_user_ptr, const int32_t **d_items,
                              int64_t *n_interactions, hipStream_t s);
  cooc::Status finish_batch(const cooc::CountResult &r, hipStream_t s, cooc_device_result *out);
  cooc::Status count_host(int64_t n_users, const int64_t *user_ptr, const int32_t *items, cooc_window_info *info);
  cooc::Status copy_batch(int64_t *row_ptr, int32_t *cols, uint32_t *cnt, int16_t *cnt16, int64_t *rowsum,
                          int32_t *rowsum32);
  cooc::Status topk_batch(int32_t topk, int32_t flags, hipStream_t s);
  // top-k into caller device buffers; d_rowsum_global (may be NULL) replaces the batch's row sums
  // (multi-GPU: the all-reduced row sums, so that k21 and the observed total are the whole log's)
  cooc::Status topk_batch_device(int32_t topk, int32_t flags, const int64_t *d_rowsum_global, int32_t *d_sizes,
                                 int32_t *d_values, double *d_scores, hipStream_t s);
  cooc::Status copy_topk_batch(int32_t *sizes, int32_t *values, double *scores);
  // row ranges of the batch result / its top-k (a JVM operator's copy-out: no single Java array holds a C3 share)
  cooc::Status copy_batch_range(int32_t r0, int32_t r1, int64_t cap, int32_t *cols, uint32_t *cnt, int16_t *cnt16);
  cooc::Status copy_topk_batch_range(int32_t r0, int32_t r1, int32_t topk, int32_t *sizes, int32_t *values,
                                     double *scores);
  cooc::Status topk_owned_host(int32_t topk, int32_t flags);
  cooc::Status comm_allgather_i64(int64_t value, int64_t *out);
  // cooc_verify_batch: invariant checks + row fingerprints of the last batch result
  cooc::Status verify_batch(int32_t flags, uint64_t *d_row_checksum, int64_t *out8, hipStream_t s);
  cooc::Status llr(int64_t n, const int64_t *k, double *out);
  cooc::Status topk_items(int32_t k, int32_t flags, int32_t n, const int32_t *items, int32_t *sizes,
                          int32_t *values, double *scores);

  // the same from host arrays (staged on the context's stream): cooc_count_owned_host
  cooc::Status count_owned_host(int64_t n_users, const int64_t *user_ptr, const int32_t *items, cooc_owned_info *info,
                                cooc_window_info *winfo);
  // multi-GPU large-universe window over the communicator (cooc_owned.hip): cooc_count_owned / cooc_topk_owned
  cooc::Status count_owned(int64_t n_users, const int64_t *d_user_ptr, const int32_t *d_items, int64_t n_interactions,
                           hipStream_t s, cooc_owned_info *info, cooc_device_result *out);
  cooc::Status topk_owned(int32_t topk, int32_t flags, int32_t *d_sizes, int32_t *d_values, double *d_scores,
                          int64_t *d_rowsum_global, hipStream_t s);

  static std::string &create_error();

  cooc_config cfg{};
  int device = 0;
  hipStream_t stream = nullptr;
  std::string last_error;
  cooc::Counter counter;
  cooc::KernelTimer timer;
  cooc::StreamState stream_state;
  cooc::Sharder sharder;
  cooc::CountResult batch_result;
  cooc::Operator op;

  // stateless batch buffers
  cooc::DevBuf b_user_ptr, b_items, b_tk_size, b_tk_val, b_tk_score, b_obs3, b_llr_terms;
  // user_cut > 0: the capped copy of a count_device CSR (first user_cut items of every user)
  cooc::DevBuf b_cut_ptr, b_cut_items, b_cut_tmp;
  cooc::DevBuf b_verify;  // cooc_verify_batch totals
  // the communicator (cooc_comm_init*) and the owned-rows exchange's buffers
  std::unique_ptr<cooc::Comm> comm;
  cooc::DevBuf own_counts, own_sort, own_tmp, own_sizes, own_owner, own_lens, own_up, own_items, own_obs, own_rowsum;
  int32_t batch_topk = 0;
  int32_t batch_topk_flags = 0;
  bool have_batch = false;
  bool batch_owned = false;  // the last batch counted only the rows of one part (cooc_count_device_owned)
  int64_t batch_observed = 0;
  int64_t batch_nnz = 0;
  // the batch result packed for range copies (once per batch): its row offsets on the host
  bool batch_packed = false;
  std::vector<int64_t> batch_rp_host;
  int64_t *batch_pk_rp = nullptr;
  int32_t *batch_pk_col = nullptr;
  uint32_t *batch_pk_cnt = nullptr;
};
