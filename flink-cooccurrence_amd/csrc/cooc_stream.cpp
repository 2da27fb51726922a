// cooc_stream.cpp — host side of the resident streaming state and of the operator mirror.
//
// StreamState restates, per tumbling window, NonSampledUserInteractionCounterOneInputStreamOperator
// .onEventTime (:113-165: expand every buffered interaction against the user's history, then
// append it), the two window aggregators (ItemRowAggregator.java:26-56, RowSumAggregator.java:
// 25-71) and ItemRowRescorerTwoInputStreamOperator.processWatermark (:116-241).  The expansion and
// reductions run on the device (cooc_count.hip); this file only keeps per-user metadata, stages
// the window's interactions and moves results.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "cooc_ctx.h"
#include "cooc_stream_kernels.h"

namespace cooc {

namespace {

// Flink TumblingEventTimeWindows.assignWindows with offset 0 [3P, Flink 1.3.2]:
// start = ts - (ts - offset + size) % size (Java remainder), maxTimestamp = start + size - 1.
int64_t window_max_ts(int64_t ts, int64_t size) {
  const int64_t start = ts - (ts + size) % size;
  return start + size - 1;
}

template <class T>
Status upload(DevBuf &b, const std::vector<T> &v, hipStream_t s) {
  COOC_TRY(b.reserve(sizeof(T) * (v.size() + 1)));
  if (!v.empty()) COOC_HIP_TRY(hipMemcpyAsync(b.p, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice, s));
  return Status::Ok();
}

// COOC_TRACE=1: per-window phase times on stderr (host wall; device phases end at a sync).
struct PhaseTrace {
  bool on = getenv("COOC_TRACE") != nullptr;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now(), last = t0;
  char buf[512];
  int len = 0;
  void mark(const char *name, hipStream_t s = nullptr) {
    if (!on) return;
    if (s) (void)hipStreamSynchronize(s);
    const auto now = std::chrono::steady_clock::now();
    len += snprintf(buf + len, sizeof(buf) - len, " %s=%.3f", name,
                    std::chrono::duration<double, std::milli>(now - last).count());
    last = now;
  }
  void done(int64_t ts) {
    if (on)
      fprintf(stderr, "[cooc] window %lld:%s total=%.3f ms\n", (long long)ts, buf,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  }
};

}  // namespace

void StreamState::release() {
  DevBuf *all[] = {&arena_,      &d_act_off_,      &d_act_len_,     &d_act_old_,   &d_cbase_,
                   &d_new_items_, &d_new_dst_ptr_, &d_new_dst_,     &d_reloc_,     &d_global_,
                   &d_grs_,       &d_touched_,     &d_scan_tmp_,    &d_scal_,      &d_topk_val_,
                   &d_topk_score_, &d_topk_size_, &d_llr_terms_, &d_lw_items_, &d_lw_up2_,
                   &d_lw_dsta_,   &d_lw_dstb_,     &d_lw_srcb_,     &d_lw_lenb_,   &d_own_base_,
                   &d_own_nnz_,   &d_rs_win_,      &d_x_nnz_,       &d_x_ent_,     &d_r_nnz_,
                   &d_r_ent_,     &d_x_h_,         &d_zero_,        &d_own_rp_,    &d_own_pcol_,
                   &d_own_pcnt_};
  for (DevBuf *b : all) b->release();
  gs_.release();
  global_ready_ = false;
  sparse_global_ = false;
}

// Keyed user state lookup (userHistoryState, NonSampled...java:129-132): a dense table for
// non-negative ids below 2^26, a hash map otherwise.
int32_t StreamState::slot_for(int32_t uid) {
  int32_t slot = -1;
  if (uid >= 0 && uid < (1 << 26)) {
    if (size_t(uid) >= dense_slot_.size()) dense_slot_.resize(std::max<size_t>(size_t(uid) + 1, dense_slot_.size() * 2), -1);
    slot = dense_slot_[uid];
  } else {
    auto it = slot_of_.find(uid);
    if (it != slot_of_.end()) slot = it->second;
  }
  if (slot >= 0) return slot;
  slot = int32_t(h_off_.size());  // userHistoryState.value() == null -> new IntArrayList(), :130-132
  if (uid >= 0 && uid < (1 << 26)) dense_slot_[uid] = slot;
  else slot_of_.emplace(uid, slot);
  h_off_.push_back(0);
  h_len_.push_back(0);
  h_cap_.push_back(0);
  staged_stamp_.push_back(-1);
  staged_pos_.push_back(0);
  return slot;
}

Status StreamState::submit(cooc_ctx &ctx, int64_t ts, int32_t n_users, const int32_t *user_ids,
                           const int64_t *user_ptr, const int32_t *items) {
  if (staged_ && ts != staged_ts_)
    return Status{COOC_ERR_STATE, "window " + std::to_string(staged_ts_) + " is staged; finish it before submitting " +
                                      std::to_string(ts)};
  const int32_t M = ctx.cfg.n_items;
  for (int32_t u = 0; u < n_users; u++) {
    if (user_ptr[u + 1] < user_ptr[u]) return Status{COOC_ERR_ARG, "user_ptr must be non-decreasing"};
    for (int64_t i = user_ptr[u]; i < user_ptr[u + 1]; i++)
      if (items[i] < 0 || items[i] >= M)
        return Status{COOC_ERR_ARG, "item id " + std::to_string(items[i]) + " outside [0, n_items)"};
  }
  const int64_t cut = ctx.cfg.user_cut;
  for (int32_t u = 0; u < n_users; u++) {
    const int32_t slot = slot_for(user_ids[u]);
    const bool staged = staged_stamp_[slot] == window_seq_;
    int64_t take = user_ptr[u + 1] - user_ptr[u];
    if (cut > 0) {
      // kMax: `userInteractions < userCut` (UserInteractionCounter...java:168) -- every accepted
      // interaction appends once to the history, so the accepted count is the history length
      const int64_t seen = int64_t(h_len_[slot]) + (staged ? int64_t(staged_items_[staged_pos_[slot]].size()) : 0);
      take = std::max<int64_t>(0, std::min<int64_t>(take, cut - seen));
      if (take == 0) continue;  // nothing of this user enters the window
    }
    int32_t j;
    if (!staged) {  // first appearance of this user in the window
      staged_stamp_[slot] = window_seq_;
      j = n_staged_++;
      staged_pos_[slot] = j;
      if (int32_t(staged_slots_.size()) < n_staged_) {
        staged_slots_.push_back(slot);
        staged_items_.emplace_back();
      } else {
        staged_slots_[j] = slot;
        staged_items_[j].clear();  // keeps the capacity of earlier windows
      }
    } else {
      j = staged_pos_[slot];
    }
    auto &dst = staged_items_[j];
    dst.insert(dst.end(), items + user_ptr[u], items + user_ptr[u] + take);
  }
  staged_ = true;
  staged_ts_ = ts;
  return Status::Ok();
}

Status StreamState::grow_arena(cooc_ctx &ctx, int64_t need) {
  if (int64_t(arena_.cap / sizeof(int32_t)) >= need) return Status::Ok();
  DevBuf bigger;
  COOC_TRY(bigger.reserve(sizeof(int32_t) * size_t(std::max<int64_t>(need, 2 * int64_t(arena_.cap / 4)))));
  if (arena_.p && arena_used_ > 0) {
    // arena_used_ already includes the new reservations; copy the whole old capacity
    COOC_HIP_TRY(hipMemcpyAsync(bigger.p, arena_.p, arena_.cap, hipMemcpyDeviceToDevice, ctx.stream));
    COOC_HIP_TRY(hipStreamSynchronize(ctx.stream));
  }
  arena_.release();
  arena_ = bigger;
  bigger.p = nullptr;
  bigger.cap = 0;
  return Status::Ok();
}

Status StreamState::ensure_global(cooc_ctx &ctx) {
  if (global_ready_) return Status::Ok();
  const int64_t M = ctx.cfg.n_items;
  if (!ctx.counter.batch_ok()) {  // large universe: sorted row slabs, grown per window
    sparse_global_ = true;
    COOC_TRY(gs_.base.reserve(sizeof(int64_t) * size_t(M)));
    COOC_TRY(gs_.len.reserve(sizeof(int32_t) * size_t(M)));
    COOC_TRY(d_grs_.reserve(sizeof(int64_t) * M));
    COOC_TRY(d_scal_.reserve(sizeof(int64_t) * 8));
    COOC_HIP_TRY(hipMemsetAsync(gs_.base.p, 0, sizeof(int64_t) * size_t(M), ctx.stream));
    COOC_HIP_TRY(hipMemsetAsync(gs_.len.p, 0, sizeof(int32_t) * size_t(M), ctx.stream));
    COOC_HIP_TRY(hipMemsetAsync(d_grs_.p, 0, sizeof(int64_t) * M, ctx.stream));
    COOC_HIP_TRY(hipMemsetAsync(d_scal_.p, 0, sizeof(int64_t) * 8, ctx.stream));
    gs_.cap = gs_.bump = gs_.live = 0;
    global_ready_ = true;
    return Status::Ok();
  }
  const size_t g_bytes = sizeof(uint32_t) * size_t(M) * size_t(M);
  size_t free_b = 0, total_b = 0;
  COOC_HIP_TRY(hipMemGetInfo(&free_b, &total_b));
  if (g_bytes > free_b / 10 * 8)
    return Status{COOC_ERR_OOM, "dense global rows need " + std::to_string(g_bytes) +
                                    " B of HBM (n_items^2 x 4); sparse global rows are not built yet"};
  COOC_TRY(d_global_.reserve(g_bytes));
  COOC_TRY(d_grs_.reserve(sizeof(int64_t) * M));
  COOC_TRY(d_scal_.reserve(sizeof(int64_t) * 8));
  COOC_HIP_TRY(hipMemsetAsync(d_global_.p, 0, g_bytes, ctx.stream));
  COOC_HIP_TRY(hipMemsetAsync(d_grs_.p, 0, sizeof(int64_t) * M, ctx.stream));
  COOC_HIP_TRY(hipMemsetAsync(d_scal_.p, 0, sizeof(int64_t) * 8, ctx.stream));
  global_ready_ = true;
  return Status::Ok();
}

Status StreamState::finish(cooc_ctx &ctx, int64_t ts, cooc_window_info *info) {
  COOC_HIP_TRY(hipSetDevice(ctx.device));
  if (staged_ && ts != staged_ts_)
    return Status{COOC_ERR_STATE, "finish_window(" + std::to_string(ts) + ") but window " +
                                      std::to_string(staged_ts_) + " is staged"};
  hipStream_t s = ctx.stream;
  const int32_t M = ctx.cfg.n_items;
  const int64_t n_act = n_staged_;
  PhaseTrace tr;
  delta_packed_ = false;  // the packed copy-out view belongs to the previous window
  empty_window_ = n_act == 0;
  // p > 1 subtasks: every subtask takes part in every window's exchange, also with no user of its own
  const bool multi = ctx.comm && ctx.comm->world() > 1;
  owned_window_ = multi;
  if (multi && empty_window_) {
    int64_t obs_total = 0;
    COOC_TRY(exchange_window(ctx, s, nullptr, 0, &obs_total));
    empty_window_ = false;
    COOC_TRY(ensure_global(ctx));
    return finish_owned(ctx, s, ts, 0, obs_total, info);
  }
  if (empty_window_) {
    // every interaction of the window was cut (user_cut): onEventTime emits nothing, no row is
    // touched and the global state is unchanged
    std::memset(&last_, 0, sizeof(last_));
    last_.ts = ts;
    last_.topk = ctx.cfg.topk;
    *info = last_;
    n_touched_ = 0;
    have_window_ = true;
    staged_ = false;
    window_seq_++;
    return Status::Ok();
  }

  // ---- host plan: history capacity (relocation on growth), append destinations, contributions
  std::vector<int64_t> act_off(n_act), cbase(n_act + 1, 0), new_ptr(n_act + 1, 0), new_dst(n_act), reloc;
  std::vector<int32_t> act_len(n_act), act_old(n_act), new_items;
  int64_t observed_window = 0;
  for (int64_t j = 0; j < n_act; j++) {
    const int32_t slot = staged_slots_[j];
    const int64_t old = h_len_[slot], w = int64_t(staged_items_[j].size());
    const int64_t need = old + w;
    if (need > int64_t(INT32_MAX)) return Status{COOC_ERR_ARG, "user history longer than 2^31"};
    if (need > h_cap_[slot]) {
      const int64_t cap = std::max<int64_t>(16, std::max<int64_t>(2 * int64_t(h_cap_[slot]), need));
      const int64_t off = arena_used_;
      arena_used_ += cap;
      if (old > 0) {
        reloc.push_back(h_off_[slot]);
        reloc.push_back(off);
        reloc.push_back(old);
      }
      h_off_[slot] = off;
      h_cap_[slot] = int32_t(std::min<int64_t>(cap, INT32_MAX));
    }
    act_off[j] = h_off_[slot];
    act_len[j] = int32_t(need);
    act_old[j] = int32_t(old);
    cbase[j + 1] = cbase[j] + need;
    new_dst[j] = h_off_[slot] + old;
    new_ptr[j + 1] = new_ptr[j] + w;
    new_items.insert(new_items.end(), staged_items_[j].begin(), staged_items_[j].end());
    observed_window += need * (need - 1) - old * (old - 1);  // sum over new positions of 2*|history|
    h_len_[slot] = int32_t(need);
  }
  tr.mark("host_plan");
  COOC_TRY(grow_arena(ctx, std::max<int64_t>(arena_used_, 1024)));
  COOC_TRY(upload(d_reloc_, reloc, s));
  COOC_TRY(upload(d_new_items_, new_items, s));
  COOC_TRY(upload(d_new_dst_ptr_, new_ptr, s));
  COOC_TRY(upload(d_new_dst_, new_dst, s));
  COOC_TRY(upload(d_act_off_, act_off, s));
  COOC_TRY(upload(d_act_len_, act_len, s));
  COOC_TRY(upload(d_act_old_, act_old, s));
  COOC_TRY(upload(d_cbase_, cbase, s));
  COOC_TRY(launch_relocate(s, int64_t(reloc.size() / 3), d_reloc_.as<int64_t>(), arena_.as<int32_t>()));
  COOC_TRY(launch_append(s, n_act, d_new_dst_ptr_.as<int64_t>(), d_new_dst_.as<int64_t>(),
                         d_new_items_.as<int32_t>(), arena_.as<int32_t>()));

  // ---- expansion + keyed reduce of the window (the hot path)
  ActiveUsers au;
  au.n_active = n_act;
  au.off = d_act_off_.as<int64_t>();
  au.len = d_act_len_.as<int32_t>();
  au.old = d_act_old_.as<int32_t>();
  au.cbase = d_cbase_.as<int64_t>();
  au.n_contrib = cbase[n_act];
  au.n_new = new_ptr[n_act];
  au.arena = arena_.as<int32_t>();
  au.arena_span = arena_used_;
  CountResult r;
  tr.mark("upload_append", s);
  if (ctx.counter.batch_ok())  // n_items < 40,320: the batch planner + k_acc_batch
    COOC_TRY(ctx.counter.run_window(au, s, &r, ctx.timer.enabled ? &ctx.timer : nullptr));  // (cooc_last_kernel_ms)
  else  // n_items >= 40,320 (or COOC_FLAG_GENERAL_PLANNER): the large-universe planner, old / new positions in one pass
    COOC_TRY(count_large_window(ctx, s, n_act, act_off, act_len, act_old, cbase[n_act], &r));
  tr.mark("count", s);

  if (multi) {  // ---- the owners' rows, then the same merge and rescoring over them
    int64_t obs_total = 0;
    COOC_TRY(exchange_window(ctx, s, &r, observed_window, &obs_total));
    COOC_TRY(ensure_global(ctx));
    return finish_owned(ctx, s, ts, observed_window, obs_total, info);
  }
  // ---- global merge + rescoring (ItemRowRescorer...java:144-228)
  COOC_TRY(ensure_global(ctx));
  int64_t *scal = d_scal_.as<int64_t>();
  COOC_TRY(launch_merge_global(s, M, r.row_base, r.row_nnz, r.col, r.cnt, r.rowsum,
                               sparse_global_ ? nullptr : d_global_.as<uint32_t>(), d_grs_.as<int64_t>(), scal,
                               observed_window));
  if (sparse_global_) {  // the window's delta rows (packed) merged into the row slabs
    int64_t *drp;
    int32_t *dcol;
    uint32_t *dcnt;
    COOC_TRY(ctx.counter.pack(s, &drp, &dcol, &dcnt));
    PlanTotals pt;
    COOC_TRY(ctx.counter.read_totals(&pt));
    int64_t new_cols = 0;
    COOC_TRY(launch_gs_merge(s, M, drp, dcol, dcnt, pt.nnz_total, gs_, d_scan_tmp_, &new_cols));
  }
  COOC_TRY(d_touched_.reserve(sizeof(int32_t) * M));
  COOC_TRY(launch_touched(s, M, r.row_nnz, d_touched_.as<int32_t>(), scal, d_scan_tmp_));
  const int32_t topk = ctx.cfg.topk;
  if (topk > 0) {
    COOC_TRY(d_topk_size_.reserve(sizeof(int32_t) * M));
    COOC_TRY(d_topk_val_.reserve(sizeof(int32_t) * size_t(M) * topk));
    COOC_TRY(d_topk_score_.reserve(sizeof(double) * size_t(M) * topk));
    if (sparse_global_)
      COOC_TRY(launch_rescore_sparse(s, d_touched_.as<int32_t>(), scal, M, gs_, d_grs_.as<int64_t>(),
                                     (ctx.cfg.flags & COOC_FLAG_EXACT_SCORES) != 0, topk, M, d_llr_terms_,
                                     d_topk_size_.as<int32_t>(), d_topk_val_.as<int32_t>(), d_topk_score_.as<double>()));
    else
      COOC_TRY(launch_rescore(s, d_touched_.as<int32_t>(), scal, M, d_global_.as<uint32_t>(), d_grs_.as<int64_t>(),
                              (ctx.cfg.flags & COOC_FLAG_EXACT_SCORES) != 0, topk, M, d_llr_terms_,
                              d_topk_size_.as<int32_t>(), d_topk_val_.as<int32_t>(), d_topk_score_.as<double>()));
  }
  tr.mark("merge_rescore", s);
  int64_t h_scal[8];
  COOC_HIP_TRY(hipMemcpyAsync(h_scal, scal, sizeof(h_scal), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  PlanTotals t;
  COOC_TRY(ctx.counter.read_totals(&t));
  if (t.err & 8) return Status{COOC_ERR_STATE, "internal bounds check failed"};
  if (t.err & 2) return Status{COOC_ERR_OVERFLOW, "a co-occurrence count exceeded uint32"};
  if (t.err & 4) return Status{COOC_ERR_OOM, "the sparse output region is exhausted"};

  n_touched_ = int32_t(h_scal[0]);
  observed_exact += observed_window;
  observed_ref = h_scal[2];
  rowsum_acc += h_scal[1];
  rescored_items += n_touched_;

  std::memset(&last_, 0, sizeof(last_));
  last_.ts = ts;
  last_.nnz = t.nnz_total;
  last_.observed = r.observed;
  last_.n_rows = n_touched_;
  last_.topk = topk;
  last_.n_topk = topk > 0 ? n_touched_ : 0;
  *info = last_;
  have_window_ = true;

  tr.done(ts);
  staged_ = false;
  n_staged_ = 0;
  window_seq_++;
  return Status::Ok();
}

// p > 1: route the window's partial delta rows (r; nullptr: this subtask has no user in the window) to their
// owners over the communicator -- row a to subtask a mod world, the keyBy(ItemCooccurrences::getItem) of
// FlinkCooccurrences.java:152 -- and merge them there (Sharder: each owned row summed in a dense LDS row, checked
// against the all-reduced row sum); the window row sums (the rowSumStream.broadcast() of :163) and the window's
// ordered pairs all-reduced.  Leaves the owned rows as an M-row view (d_own_base_, d_own_nnz_, own_col_/cnt_)
// and every item's window row sum in d_rs_win_.
Status StreamState::exchange_window(cooc_ctx &ctx, hipStream_t s, const CountResult *r, int64_t obs_local,
                                    int64_t *obs_total) {
  Comm &c = *ctx.comm;
  const int32_t M = ctx.cfg.n_items, W = c.world(), part = c.rank();
  auto rows_owned = [&](int32_t q) { return int64_t(M > q ? (M - q + W - 1) / W : 0); };
  CountResult zero;
  if (!r) {  // no user here: zero partial rows
    COOC_TRY(d_zero_.reserve(sizeof(int64_t) * size_t(M) * 2 + 64));
    COOC_HIP_TRY(hipMemsetAsync(d_zero_.p, 0, sizeof(int64_t) * size_t(M) * 2 + 64, s));
    zero.row_base = d_zero_.as<int64_t>();
    zero.rowsum = d_zero_.as<int64_t>() + M;
    zero.row_nnz = reinterpret_cast<int32_t *>(d_zero_.as<int64_t>());
    zero.col = reinterpret_cast<int32_t *>(d_zero_.as<int64_t>());
    zero.cnt = reinterpret_cast<uint32_t *>(d_zero_.as<int64_t>());
    r = &zero;
  }
  // 1. entries per owner, the owner-major row counts and entries; every subtask's counts all-gathered
  std::vector<int64_t> h_ent(W), H(size_t(W) * W);
  COOC_TRY(ctx.sharder.plan(*r, M, W, s, h_ent.data()));
  int64_t n_send = 0;
  for (int64_t v : h_ent) n_send += v;
  COOC_TRY(d_x_nnz_.reserve(sizeof(int32_t) * size_t(M) + 4));
  COOC_TRY(d_x_ent_.reserve(sizeof(uint64_t) * size_t(n_send + 1)));
  COOC_TRY(ctx.sharder.pack(*r, M, W, s, d_x_nnz_.as<int32_t>(), n_send ? d_x_ent_.as<uint64_t>() : nullptr));
  COOC_TRY(d_x_h_.reserve(sizeof(int64_t) * size_t(W) * (W + 1)));
  int64_t *dh = d_x_h_.as<int64_t>();
  COOC_HIP_TRY(hipMemcpyAsync(dh, h_ent.data(), sizeof(int64_t) * W, hipMemcpyHostToDevice, s));
  COOC_TRY(c.allgather(dh, dh + W, sizeof(int64_t) * W, s));
  COOC_HIP_TRY(hipMemcpyAsync(H.data(), dh + W, sizeof(int64_t) * W * W, hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  // 2. row counts and entries to their owners (every peer pair in one exchange)
  const int64_t R = rows_owned(part);
  std::vector<int64_t> so(W), sb(W), ro(W), rb(W);
  int64_t off = 0;
  for (int32_t q = 0; q < W; q++) {
    so[q] = off;
    sb[q] = sizeof(int32_t) * rows_owned(q);
    off += sb[q];
    ro[q] = int64_t(sizeof(int32_t)) * q * R;
    rb[q] = int64_t(sizeof(int32_t)) * R;
  }
  COOC_TRY(d_r_nnz_.reserve(sizeof(int32_t) * size_t(W * R) + 4));
  COOC_TRY(c.alltoallv(d_x_nnz_.p, so.data(), sb.data(), d_r_nnz_.p, ro.data(), rb.data(), s));
  int64_t n_recv = 0;
  off = 0;
  for (int32_t q = 0; q < W; q++) {
    so[q] = off;
    sb[q] = int64_t(sizeof(uint64_t)) * h_ent[q];
    off += sb[q];
    ro[q] = int64_t(sizeof(uint64_t)) * n_recv;
    rb[q] = int64_t(sizeof(uint64_t)) * H[size_t(q) * W + part];
    n_recv += H[size_t(q) * W + part];
  }
  COOC_TRY(d_r_ent_.reserve(sizeof(uint64_t) * size_t(n_recv + 1)));
  COOC_TRY(c.alltoallv(d_x_ent_.p, so.data(), sb.data(), d_r_ent_.p, ro.data(), rb.data(), s));
  // 3. the window row sums of every item and the window's pairs, all-reduced
  COOC_TRY(d_rs_win_.reserve(sizeof(int64_t) * (size_t(M) + 1)));
  int64_t *rs = d_rs_win_.as<int64_t>();
  COOC_HIP_TRY(hipMemcpyAsync(rs, r->rowsum, sizeof(int64_t) * size_t(M), hipMemcpyDeviceToDevice, s));
  COOC_HIP_TRY(hipMemcpyAsync(rs + M, &obs_local, sizeof(int64_t), hipMemcpyHostToDevice, s));
  COOC_TRY(c.allreduce_sum_i64(rs, M + 1, s));
  COOC_HIP_TRY(hipMemcpyAsync(obs_total, rs + M, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  // 4. the owned rows merged (checked against the all-reduced row sums), as an M-row view
  MergeResult m;
  COOC_TRY(ctx.sharder.merge(M, W, part, d_r_nnz_.as<int32_t>(), d_r_ent_.as<uint64_t>(), rs, s, &m));
  COOC_TRY(d_own_base_.reserve(sizeof(int64_t) * size_t(M)));
  COOC_TRY(d_own_nnz_.reserve(sizeof(int32_t) * size_t(M)));
  COOC_TRY(launch_owned_view(s, M, W, part, m.n_rows, m.row_base, m.row_nnz, d_own_base_.as<int64_t>(),
                             d_own_nnz_.as<int32_t>()));
  own_col_ = m.col;
  own_cnt_ = m.cnt;
  COOC_HIP_TRY(hipStreamSynchronize(s));
  return Status::Ok();
}

// p > 1: the owned delta rows merged into the resident rows, every item's row sum into the global row sums, the
// owned touched rows rescored; the window's outputs are this subtask's owned rows (each item on one subtask).
Status StreamState::finish_owned(cooc_ctx &ctx, hipStream_t s, int64_t ts, int64_t obs_local, int64_t obs_total,
                                 cooc_window_info *info) {
  const int32_t M = ctx.cfg.n_items;
  int64_t *scal = d_scal_.as<int64_t>();
  COOC_TRY(launch_merge_owned(s, M, d_own_base_.as<int64_t>(), d_own_nnz_.as<int32_t>(), own_col_, own_cnt_,
                              d_rs_win_.as<int64_t>(), sparse_global_ ? nullptr : d_global_.as<uint32_t>(),
                              d_grs_.as<int64_t>(), scal, obs_total));
  int64_t nnz = 0;
  // the owned delta rows packed (M-row CSR, ascending columns): the window's output, and for a large universe the
  // delta merged into the resident row slabs (ItemRowRescorer...java:171-177)
  COOC_TRY(launch_pack_rows(s, M, d_own_base_.as<int64_t>(), d_own_nnz_.as<int32_t>(), own_col_, own_cnt_, d_own_rp_,
                            d_own_pcol_, d_own_pcnt_, d_scan_tmp_, &nnz));  // (synchronises s)
  if (sparse_global_) {
    int64_t new_cols = 0;
    COOC_TRY(launch_gs_merge(s, M, d_own_rp_.as<int64_t>(), d_own_pcol_.as<int32_t>(), d_own_pcnt_.as<uint32_t>(), nnz,
                             gs_, d_scan_tmp_, &new_cols));
  }
  COOC_TRY(d_touched_.reserve(sizeof(int32_t) * M));
  COOC_TRY(launch_touched(s, M, d_own_nnz_.as<int32_t>(), d_touched_.as<int32_t>(), scal, d_scan_tmp_));
  const int32_t topk = ctx.cfg.topk;
  if (topk > 0) {
    COOC_TRY(d_topk_size_.reserve(sizeof(int32_t) * M));
    COOC_TRY(d_topk_val_.reserve(sizeof(int32_t) * size_t(M) * topk));
    COOC_TRY(d_topk_score_.reserve(sizeof(double) * size_t(M) * topk));
    if (sparse_global_)
      COOC_TRY(launch_rescore_sparse(s, d_touched_.as<int32_t>(), scal, M, gs_, d_grs_.as<int64_t>(),
                                     (ctx.cfg.flags & COOC_FLAG_EXACT_SCORES) != 0, topk, M, d_llr_terms_,
                                     d_topk_size_.as<int32_t>(), d_topk_val_.as<int32_t>(), d_topk_score_.as<double>()));
    else
      COOC_TRY(launch_rescore(s, d_touched_.as<int32_t>(), scal, M, d_global_.as<uint32_t>(), d_grs_.as<int64_t>(),
                              (ctx.cfg.flags & COOC_FLAG_EXACT_SCORES) != 0, topk, M, d_llr_terms_,
                              d_topk_size_.as<int32_t>(), d_topk_val_.as<int32_t>(), d_topk_score_.as<double>()));
  }
  int64_t h_scal[8];
  COOC_HIP_TRY(hipMemcpyAsync(h_scal, scal, sizeof(h_scal), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  PlanTotals t;
  COOC_TRY(ctx.counter.read_totals(&t));
  if (t.err & 8) return Status{COOC_ERR_STATE, "internal bounds check failed"};
  if (t.err & 2) return Status{COOC_ERR_OVERFLOW, "a co-occurrence count exceeded uint32"};
  n_touched_ = int32_t(h_scal[0]);
  observed_exact += obs_local;  // this subtask's users' pairs (the rescorer's total, observed_ref, is the job's)
  observed_ref = h_scal[2];
  rowsum_acc += h_scal[4];      // this subtask's owned row sums: the p accumulators sum to the job's
  rescored_items += n_touched_;
  std::memset(&last_, 0, sizeof(last_));
  last_.ts = ts;
  last_.nnz = nnz;
  last_.observed = obs_local;   // this subtask's users' pairs: the p accumulators sum to the job's
  last_.n_rows = n_touched_;
  last_.topk = topk;
  last_.n_topk = topk > 0 ? n_touched_ : 0;
  *info = last_;
  have_window_ = true;
  staged_ = false;
  n_staged_ = 0;
  window_seq_++;
  return Status::Ok();
}

Status StreamState::count_large_window(cooc_ctx &ctx, hipStream_t s, int64_t n_act, const std::vector<int64_t> &act_off,
                                      const std::vector<int32_t> &act_len, const std::vector<int32_t> &act_old,
                                      int64_t n_full, CountResult *r) {
  // every pair whose later position is new (NonSampled...java:129-161), in one pass: user j's lists A_j
  // (its whole history) and B_j (the window's items, the tail of A_j) side by side; a new position
  // walks A_j, an old one B_j (run_sparse's SparseWindow, k_sp_window_contribs): 2 new |A_j| pair work
  // per user instead of |A_j|^2 + |old|^2
  std::vector<int64_t> up2(2 * n_act + 1), dst_a(n_act), dst_b(n_act), src_b(n_act);
  std::vector<int32_t> len_b(n_act);
  int64_t o = 0;
  for (int64_t j = 0; j < n_act; j++) {
    up2[2 * j] = dst_a[j] = o;
    o += act_len[j];
    up2[2 * j + 1] = dst_b[j] = o;
    src_b[j] = act_off[j] + act_old[j];
    len_b[j] = act_len[j] - act_old[j];
    o += len_b[j];
  }
  up2[2 * n_act] = o;
  COOC_TRY(upload(d_lw_up2_, up2, s));
  COOC_TRY(upload(d_lw_dsta_, dst_a, s));
  COOC_TRY(upload(d_lw_dstb_, dst_b, s));
  COOC_TRY(upload(d_lw_srcb_, src_b, s));
  COOC_TRY(upload(d_lw_lenb_, len_b, s));
  COOC_TRY(d_lw_items_.reserve(sizeof(int32_t) * size_t(std::max<int64_t>(o, 1))));
  int32_t *lists = d_lw_items_.as<int32_t>();
  COOC_TRY(launch_gather_lists(s, n_act, d_act_off_.as<int64_t>(), d_act_len_.as<int32_t>(), d_lw_dsta_.as<int64_t>(),
                               arena_.as<int32_t>(), lists));
  COOC_TRY(launch_gather_lists(s, n_act, d_lw_srcb_.as<int64_t>(), d_lw_lenb_.as<int32_t>(), d_lw_dstb_.as<int64_t>(),
                               arena_.as<int32_t>(), lists));
  SparseWindow w;
  w.n_users = n_act;
  w.old = d_act_old_.as<int32_t>();
  w.cbase = d_cbase_.as<int64_t>();
  w.n_contrib = n_full;
  return ctx.counter.run_sparse(2 * n_act, d_lw_up2_.as<int64_t>(), lists, o, s, r,
                                ctx.timer.enabled ? &ctx.timer : nullptr, nullptr, 0, nullptr, 0, &w);
}

Status StreamState::copy_delta(cooc_ctx &ctx, int32_t *rows, int64_t *row_ptr, int32_t *cols, uint32_t *cnt,
                               int16_t *cnt16) {
  if (!have_window_) return Status{COOC_ERR_STATE, "no finished window"};
  COOC_HIP_TRY(hipSetDevice(ctx.device));
  if (empty_window_) {
    if (row_ptr) row_ptr[0] = 0;
    return Status::Ok();
  }
  COOC_TRY(pack_delta(ctx));
  const int32_t R = int32_t(delta_rows_.size());
  if (rows) std::memcpy(rows, delta_rows_.data(), sizeof(int32_t) * R);
  if (row_ptr) std::memcpy(row_ptr, delta_start_.data(), sizeof(int64_t) * (R + 1));
  return copy_entries(0, delta_start_[R], cols, cnt, cnt16);
}

// The window's delta rows packed (contiguous, ascending row then column) once per window, with the
// host list of rows that have entries and their starts in the packed arrays.
Status StreamState::pack_delta(cooc_ctx &ctx) {
  if (delta_packed_) return Status::Ok();
  const int32_t M = ctx.cfg.n_items;
  if (owned_window_) {  // (packed by finish_owned)
    pk_rp_ = d_own_rp_.as<int64_t>();
    pk_col_ = d_own_pcol_.as<int32_t>();
    pk_cnt_ = d_own_pcnt_.as<uint32_t>();
  } else {
    COOC_TRY(ctx.counter.pack(ctx.stream, &pk_rp_, &pk_col_, &pk_cnt_));
  }
  COOC_HIP_TRY(hipStreamSynchronize(ctx.stream));
  std::vector<int64_t> rp(M + 1);
  COOC_HIP_TRY(hipMemcpy(rp.data(), pk_rp_, sizeof(int64_t) * (M + 1), hipMemcpyDeviceToHost));
  delta_rows_.clear();
  delta_start_.clear();
  for (int32_t a = 0; a < M; a++) {
    if (rp[a + 1] == rp[a]) continue;
    delta_rows_.push_back(a);
    delta_start_.push_back(rp[a]);
  }
  delta_start_.push_back(rp[M]);
  delta_packed_ = true;
  return Status::Ok();
}

Status StreamState::copy_entries(int64_t e0, int64_t e1, int32_t *cols, uint32_t *cnt, int16_t *cnt16) {
  const int64_t n = e1 - e0;
  if (n <= 0) return Status::Ok();
  if (cols) COOC_HIP_TRY(hipMemcpy(cols, pk_col_ + e0, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
  if (cnt || cnt16) {
    std::vector<uint32_t> tmp;
    uint32_t *dst = cnt;
    if (!dst) {
      tmp.resize(n);
      dst = tmp.data();
    }
    COOC_HIP_TRY(hipMemcpy(dst, pk_cnt_ + e0, sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
    if (cnt16)  // ItemRowAggregator's Int2ShortOpenHashMap value (short addTo wraps)
      for (int64_t i = 0; i < n; i++) cnt16[i] = int16_t(uint16_t(dst[i]));
  }
  return Status::Ok();
}

Status StreamState::copy_delta_range(cooc_ctx &ctx, int32_t r0, int32_t r1, int64_t cap, int32_t *cols,
                                     uint32_t *cnt, int16_t *cnt16) {
  if (!have_window_) return Status{COOC_ERR_STATE, "no finished window"};
  COOC_HIP_TRY(hipSetDevice(ctx.device));
  const int32_t R = empty_window_ ? 0 : last_.n_rows;
  if (r0 < 0 || r1 < r0 || r1 > R)
    return Status{COOC_ERR_ARG, "delta rows [" + std::to_string(r0) + ", " + std::to_string(r1) + ") outside [0, " +
                                    std::to_string(R) + ")"};
  if (r0 == r1) return Status::Ok();
  COOC_TRY(pack_delta(ctx));
  const int64_t n = delta_start_[r1] - delta_start_[r0];
  if ((cols || cnt || cnt16) && n > cap)  // (the caller's buffers are smaller than the range)
    return Status{COOC_ERR_ARG, "delta rows [" + std::to_string(r0) + ", " + std::to_string(r1) + ") hold " +
                                    std::to_string(n) + " entries, more than the " + std::to_string(cap) + " given"};
  return copy_entries(delta_start_[r0], delta_start_[r1], cols, cnt, cnt16);
}

Status StreamState::copy_rowsums(cooc_ctx &ctx, int32_t *items, int64_t *delta, int32_t *delta32) {
  if (!have_window_) return Status{COOC_ERR_STATE, "no finished window"};
  if (empty_window_) return Status::Ok();
  COOC_HIP_TRY(hipSetDevice(ctx.device));
  const int32_t M = ctx.cfg.n_items;
  std::vector<int32_t> nnz(M);
  std::vector<int64_t> rs(M);
  // (p > 1: the owned rows with a delta and their all-reduced row sums: each item on its owner only)
  COOC_HIP_TRY(hipMemcpy(nnz.data(), owned_window_ ? d_own_nnz_.as<int32_t>() : ctx.counter.last_row_nnz(),
                         sizeof(int32_t) * M, hipMemcpyDeviceToHost));
  COOC_HIP_TRY(hipMemcpy(rs.data(), owned_window_ ? d_rs_win_.as<int64_t>() : ctx.counter.last_rowsum(),
                         sizeof(int64_t) * M, hipMemcpyDeviceToHost));
  int32_t k = 0;
  for (int32_t a = 0; a < M; a++) {
    if (nnz[a] == 0) continue;
    if (items) items[k] = a;
    if (delta) delta[k] = rs[a];
    if (delta32) delta32[k] = int32_t(uint32_t(uint64_t(rs[a])));  // Java int accumulation
    k++;
  }
  return Status::Ok();
}

Status StreamState::copy_topk(cooc_ctx &ctx, int32_t *rows, int32_t *sizes, int32_t *values, double *scores) {
  if (!have_window_) return Status{COOC_ERR_STATE, "no finished window"};
  if (ctx.cfg.topk <= 0) return Status{COOC_ERR_STATE, "rescoring is disabled (topk == 0)"};
  COOC_HIP_TRY(hipSetDevice(ctx.device));
  const size_t n = size_t(n_touched_), k = size_t(ctx.cfg.topk);
  if (n == 0) return Status::Ok();
  if (rows) COOC_HIP_TRY(hipMemcpy(rows, d_touched_.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
  if (sizes) COOC_HIP_TRY(hipMemcpy(sizes, d_topk_size_.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
  if (values) COOC_HIP_TRY(hipMemcpy(values, d_topk_val_.p, sizeof(int32_t) * n * k, hipMemcpyDeviceToHost));
  if (scores) COOC_HIP_TRY(hipMemcpy(scores, d_topk_score_.p, sizeof(double) * n * k, hipMemcpyDeviceToHost));
  return Status::Ok();
}

Status StreamState::global_rowsums(cooc_ctx &ctx, int64_t *exact, int32_t *v32) {
  const int32_t M = ctx.cfg.n_items;
  std::vector<int64_t> rs(M, 0);
  if (global_ready_) {
    COOC_HIP_TRY(hipSetDevice(ctx.device));
    COOC_HIP_TRY(hipMemcpy(rs.data(), d_grs_.p, sizeof(int64_t) * M, hipMemcpyDeviceToHost));
  }
  if (exact) std::memcpy(exact, rs.data(), sizeof(int64_t) * M);
  if (v32)  // globalItemRowSums (Int2IntOpenHashMap, int32 wrap)
    for (int32_t a = 0; a < M; a++) v32[a] = int32_t(uint32_t(uint64_t(rs[a])));
  return Status::Ok();
}

Status StreamState::global_row_nnz(cooc_ctx &ctx, int32_t item, int64_t *nnz) {
  const int32_t M = ctx.cfg.n_items;
  if (item < 0 || item >= M) return Status{COOC_ERR_ARG, "item outside [0, n_items)"};
  *nnz = 0;
  if (!global_ready_) return Status::Ok();
  COOC_HIP_TRY(hipSetDevice(ctx.device));
  if (sparse_global_) {
    int32_t n = 0;
    COOC_HIP_TRY(hipMemcpy(&n, gs_.len.as<int32_t>() + item, sizeof(int32_t), hipMemcpyDeviceToHost));
    *nnz = n;
    return Status::Ok();
  }
  std::vector<uint32_t> row(M);
  COOC_HIP_TRY(hipMemcpy(row.data(), d_global_.as<uint32_t>() + int64_t(item) * M, sizeof(uint32_t) * M,
                         hipMemcpyDeviceToHost));
  *nnz = std::count_if(row.begin(), row.end(), [](uint32_t v) { return v != 0; });
  return Status::Ok();
}

Status StreamState::global_row(cooc_ctx &ctx, int32_t item, int32_t *cols, uint32_t *cnt, int16_t *cnt16) {
  const int32_t M = ctx.cfg.n_items;
  if (item < 0 || item >= M) return Status{COOC_ERR_ARG, "item outside [0, n_items)"};
  if (!global_ready_) return Status::Ok();
  COOC_HIP_TRY(hipSetDevice(ctx.device));
  if (sparse_global_) {
    int32_t n = 0;
    int64_t b = 0;
    COOC_HIP_TRY(hipMemcpy(&n, gs_.len.as<int32_t>() + item, sizeof(int32_t), hipMemcpyDeviceToHost));
    COOC_HIP_TRY(hipMemcpy(&b, gs_.base.as<int64_t>() + item, sizeof(int64_t), hipMemcpyDeviceToHost));
    std::vector<uint32_t> c(n);
    if (n && cols) COOC_HIP_TRY(hipMemcpy(cols, gs_.col.as<int32_t>() + b, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    if (n) COOC_HIP_TRY(hipMemcpy(c.data(), gs_.cnt.as<uint32_t>() + b, sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
    for (int32_t i = 0; i < n; i++) {
      if (cnt) cnt[i] = c[i];
      if (cnt16) cnt16[i] = int16_t(uint16_t(c[i]));
    }
    return Status::Ok();
  }
  std::vector<uint32_t> row(M);
  COOC_HIP_TRY(hipMemcpy(row.data(), d_global_.as<uint32_t>() + int64_t(item) * M, sizeof(uint32_t) * M,
                         hipMemcpyDeviceToHost));
  int64_t k = 0;
  for (int32_t b = 0; b < M; b++) {
    if (!row[b]) continue;  // a key exists iff it was ever touched (all increments are +1)
    if (cols) cols[k] = b;
    if (cnt) cnt[k] = row[b];
    if (cnt16) cnt16[k] = int16_t(uint16_t(row[b]));
    k++;
  }
  return Status::Ok();
}

// ---- NonSampledUserInteractionCounterOneInputStreamOperator mirror -------------------------------
Status Operator::process_elements(cooc_ctx &ctx, int64_t n, const int32_t *users, const int32_t *items,
                                  const int64_t *ts, int64_t *n_late) {
  const int32_t M = ctx.cfg.n_items;
  int64_t late = 0;
  for (int64_t i = 0; i < n; i++) {
    if (ts[i] <= watermark) {  // :89-91
      late++;
      continue;
    }
    if (items[i] < 0 || items[i] >= M)
      return Status{COOC_ERR_ARG, "item id " + std::to_string(items[i]) + " outside [0, n_items)"};
    Pending &p = pending_[window_max_ts(ts[i], ctx.cfg.window_size_ms)];  // :93-100
    p.users.push_back(users[i]);
    p.items.push_back(items[i]);
  }
  late_elements += late;
  if (n_late) *n_late = late;
  return Status::Ok();
}

Status Operator::process_watermark(cooc_ctx &ctx, int64_t wm, int32_t *fired, cooc_window_info *info) {
  if (wm > watermark) watermark = wm;
  *fired = 0;
  if (ctx.comm && ctx.comm->world() > 1) {
    // p > 1: Flink does not hand every subtask the same watermarks (each is the minimum over its own input
    // channels, which arrive in their own order), so what fires is decided from all-gathered state only.  An
    // agreement step all-gathers (this subtask's watermark, its earliest pending window); agreed_ becomes the
    // minimum watermark -- every window ending at or before it is complete on every subtask, a record of it
    // arriving later being late everywhere (:89-91) -- and the earliest pending window ending there fires on
    // every subtask together (one without records in it joins with no user).  A subtask runs a step while its
    // own watermark is ahead of agreed_ (it waits there for the others to catch up) and after a step that fired
    // (more windows may be due): both conditions are functions of the all-gathered state and of watermarks that
    // only grow, so every subtask runs the same sequence of collectives whatever order its watermarks came in.
    const int world = ctx.comm->world();
    std::vector<int64_t> all(static_cast<size_t>(world));
    while (regather_ || watermark > agreed_) {
      regather_ = false;
      COOC_TRY(ctx.comm_allgather_i64(watermark, all.data()));
      const int64_t wmin = *std::min_element(all.begin(), all.end());
      const int64_t mine = pending_.empty() ? INT64_MAX : pending_.begin()->first;
      COOC_TRY(ctx.comm_allgather_i64(mine, all.data()));
      if (wmin > agreed_) agreed_ = wmin;
      const int64_t due = *std::min_element(all.begin(), all.end());
      if (due != INT64_MAX && due <= agreed_) {
        regather_ = true;
        return fire(ctx, due, mine == due, fired, info);
      }
    }
    return Status::Ok();
  }
  auto it = pending_.begin();
  if (it == pending_.end() || it->first > watermark) return Status::Ok();
  return fire(ctx, it->first, true, fired, info);
}

// onEventTime for every user of the window max_ts (mine: this subtask holds its records, the earliest pending
// window; else it joins the p > 1 exchange with no user).
Status Operator::fire(cooc_ctx &ctx, int64_t max_ts, bool mine, int32_t *fired, cooc_window_info *info) {
  if (!mine) {
    COOC_TRY(ctx.stream_state.finish(ctx, max_ts, info));
    *fired = 1;
    return Status::Ok();
  }
  // group the buffered interactions by user, keeping each user's arrival order (windowState list order, :118)
  auto it = pending_.begin();
  Pending &p = it->second;
  std::unordered_map<int32_t, int32_t> idx;
  std::vector<int32_t> uids;
  std::vector<int64_t> counts;
  std::vector<int32_t> which(p.users.size());
  for (size_t i = 0; i < p.users.size(); i++) {
    auto f = idx.find(p.users[i]);
    int32_t j;
    if (f == idx.end()) {
      j = int32_t(uids.size());
      idx.emplace(p.users[i], j);
      uids.push_back(p.users[i]);
      counts.push_back(0);
    } else {
      j = f->second;
    }
    which[i] = j;
    counts[j]++;
  }
  std::vector<int64_t> ptr(uids.size() + 1, 0);
  for (size_t j = 0; j < uids.size(); j++) ptr[j + 1] = ptr[j] + counts[j];
  std::vector<int64_t> fill(ptr.begin(), ptr.end() - 1);
  std::vector<int32_t> grouped(p.items.size());
  for (size_t i = 0; i < p.items.size(); i++) grouped[fill[which[i]]++] = p.items[i];
  COOC_TRY(ctx.stream_state.submit(ctx, max_ts, int32_t(uids.size()), uids.data(), ptr.data(), grouped.data()));
  pending_.erase(it);
  COOC_TRY(ctx.stream_state.finish(ctx, max_ts, info));
  *fired = 1;
  return Status::Ok();
}

}  // namespace cooc
