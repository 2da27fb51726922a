// cooc_ctx.cpp — context lifecycle and the stateless one-window batch entry points.
#include "cooc_ctx.h"
#include "cooc_stream_kernels.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

using cooc::Status;

std::string &cooc_ctx::create_error() {
  static thread_local std::string e;
  return e;
}

Status cooc_ctx::init(const cooc_config &c) {
  cfg = c;
  if (c.n_items <= 0) return Status{COOC_ERR_ARG, "n_items must be > 0"};
  if (c.topk < 0 || c.topk > 32767)  // topK is a Java short (Configuration.java:153, ItemRowRescorer...java:31)
    return Status{COOC_ERR_ARG, std::to_string(c.topk) + " is not a valid topK"};
  if (c.window_size_ms <= 0) return Status{COOC_ERR_ARG, "window size must be > 0"};
  if (c.user_cut < 0 || c.user_cut > 32767)  // userCut is a Java short (UserInteractionCounter...java:54,76)
    return Status{COOC_ERR_ARG, std::to_string(c.user_cut) + " is not a valid userCut"};
  int n_dev = 0;
  hipError_t e = hipGetDeviceCount(&n_dev);
  if (e != hipSuccess || n_dev == 0) {
    (void)hipGetLastError();
    return Status{COOC_ERR_HIP, "no HIP device available (the co-occurrence core has no CPU fallback)"};
  }
  if (c.device >= n_dev) return Status{COOC_ERR_ARG, "device ordinal out of range"};
  if (c.device >= 0) COOC_HIP_TRY(hipSetDevice(c.device));
  COOC_HIP_TRY(hipGetDevice(&device));
  COOC_HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  COOC_HIP_TRY(hipEventCreate(&timer.acc_begin));
  COOC_HIP_TRY(hipEventCreate(&timer.acc_end));
  COOC_TRY(counter.init(c.n_items));
  counter.set_output_layout((c.flags & COOC_FLAG_OUTPUT_DENSE) ? 2 : (c.flags & COOC_FLAG_OUTPUT_CSR) ? 1 : 0);
  counter.set_general_only((c.flags & COOC_FLAG_GENERAL_PLANNER) != 0);
  counter.set_sort_rows((c.flags & COOC_FLAG_SORT_ROWS) != 0);
  counter.set_relabel((c.flags & COOC_FLAG_COLUMN_ORDER) == 0);
  counter.set_any_order((c.flags & COOC_FLAG_ANY_ORDER) != 0);
  return Status::Ok();
}

cooc_ctx::~cooc_ctx() {
  (void)hipSetDevice(device);
  if (stream) (void)hipStreamSynchronize(stream);
  stream_state.release();
  sharder.release();
  counter.release();
  comm.reset();
  cooc::DevBuf *bufs[] = {&b_user_ptr, &b_items, &b_tk_size, &b_tk_val, &b_tk_score, &b_obs3,
                          &b_cut_ptr, &b_cut_items, &b_cut_tmp, &b_llr_terms, &b_verify,
                          &own_counts, &own_sort, &own_tmp, &own_sizes, &own_owner, &own_lens,
                          &own_up, &own_items, &own_obs, &own_rowsum};
  for (auto *b : bufs) b->release();
  if (timer.acc_begin) (void)hipEventDestroy(timer.acc_begin);
  if (timer.acc_end) (void)hipEventDestroy(timer.acc_end);
  if (stream) (void)hipStreamDestroy(stream);
}

Status cooc_ctx::count_device(int64_t n_users, const int64_t *d_user_ptr, const int32_t *d_items,
                              int64_t n_interactions, hipStream_t s, cooc_device_result *out) {
  COOC_HIP_TRY(hipSetDevice(device));
  have_batch = false;
  batch_topk = 0;
  COOC_TRY(apply_user_cut(n_users, &d_user_ptr, &d_items, &n_interactions, s));
  batch_owned = false;
  cooc::CountResult r;
  if (counter.batch_ok()) {
    COOC_TRY(counter.run_batch(n_users, d_user_ptr, d_items, n_interactions, s, &r, timer.enabled ? &timer : nullptr));
  } else {
    COOC_TRY(counter.run_sparse(n_users, d_user_ptr, d_items, n_interactions, s, &r, timer.enabled ? &timer : nullptr));
  }
  return finish_batch(r, s, out);
}

Status cooc_ctx::count_device_owned(int64_t n_users, const int64_t *d_user_ptr, const int32_t *d_items,
                                    int64_t n_interactions, const int32_t *d_owner, int32_t part,
                                    const int64_t *d_item_counts, int64_t n_total, hipStream_t s,
                                    cooc_device_result *out) {
  if (!counter.sparse())
    return Status{COOC_ERR_ARG, "cooc_count_device_owned needs n_items >= " + std::to_string(cooc::Counter::kBatchMaxItems) +
                                    " (smaller universes shard with cooc_shard_plan / cooc_shard_count)"};
  COOC_HIP_TRY(hipSetDevice(device));
  have_batch = false;
  batch_topk = 0;
  COOC_TRY(apply_user_cut(n_users, &d_user_ptr, &d_items, &n_interactions, s));
  cooc::CountResult r;
  COOC_TRY(counter.run_sparse(n_users, d_user_ptr, d_items, n_interactions, s, &r, timer.enabled ? &timer : nullptr,
                              d_owner, part, d_item_counts, n_total));
  COOC_TRY(finish_batch(r, s, out));
  batch_owned = true;
  return Status::Ok();
}

Status cooc_ctx::apply_user_cut(int64_t n_users, const int64_t **d_user_ptr, const int32_t **d_items,
                                int64_t *n_interactions, hipStream_t s) {
  if (cfg.user_cut <= 0) return Status::Ok();
  // kMax (UserInteractionCounter...java:168): only the first user_cut items of every user are
  // expanded; one capping pass over the CSR, then the same path on the capped copy
  COOC_TRY(b_cut_ptr.reserve(sizeof(int64_t) * size_t(n_users + 1)));
  COOC_TRY(b_cut_items.reserve(sizeof(int32_t) * size_t(std::max<int64_t>(*n_interactions, 1))));
  int64_t n_cut = 0;
  COOC_TRY(cooc::launch_user_cut(s, n_users, *d_user_ptr, *d_items, cfg.user_cut, b_cut_ptr.as<int64_t>(),
                                 b_cut_items.as<int32_t>(), b_cut_tmp, &n_cut));
  *d_user_ptr = b_cut_ptr.as<int64_t>();
  *d_items = b_cut_items.as<int32_t>();
  *n_interactions = n_cut;
  return Status::Ok();
}

cooc::Status cooc_ctx::finish_batch(const cooc::CountResult &r, hipStream_t s, cooc_device_result *out) {
  COOC_HIP_TRY(hipStreamSynchronize(s));
  // totals (nnz, overflow flag) are written by the last kernels of the run
  int64_t nnz = 0, err = 0, bad_row = -1;
  {
    cooc::PlanTotals h;
    COOC_TRY(counter.read_totals(&h));
    nnz = h.nnz_total;
    err = h.err;
    bad_row = counter.sparse() ? h.bad_row : -1;
  }
  if (err & 8)
    return Status{COOC_ERR_STATE, "internal bounds check failed" + (bad_row >= 0 ? " (row " + std::to_string(bad_row) + ")" : std::string())};
  if (err & 2)
    return Status{COOC_ERR_OVERFLOW, "row-sum check failed" + (bad_row >= 0 ? " (row " + std::to_string(bad_row) + ")" : std::string()) +
                                         ": a row's exact counts do not add up to its closed-form row sum (a co-occurrence "
                                         "count exceeded uint32)"};
  if (err & 4) return Status{COOC_ERR_OOM, "the sparse output region is exhausted"};
  out->n_items = cfg.n_items;
  out->nnz = nnz;
  out->observed = r.observed;
  out->row_base = r.row_base;
  out->row_nnz = r.row_nnz;
  out->col = r.col;
  out->cnt = r.cnt;
  out->rowsum = r.rowsum;
  out->dense = r.dense;
  have_batch = true;
  batch_packed = false;
  batch_result = r;
  batch_result.nnz = nnz;
  batch_observed = r.observed;
  batch_nnz = nnz;
  return Status::Ok();
}

Status cooc_ctx::count_host(int64_t n_users, const int64_t *user_ptr, const int32_t *items, cooc_window_info *info) {
  COOC_HIP_TRY(hipSetDevice(device));
  if (user_ptr && n_users > 0 && user_ptr[0] != 0) return Status{COOC_ERR_ARG, "user_ptr[0] must be 0"};
  for (int64_t u = 0; u < n_users; u++)
    if (user_ptr[u + 1] < user_ptr[u]) return Status{COOC_ERR_ARG, "user_ptr must be non-decreasing"};
  const int64_t n = n_users > 0 ? user_ptr[n_users] : 0;
  if (n > 0 && !items) return Status{COOC_ERR_ARG, "items is NULL"};
  COOC_TRY(b_user_ptr.reserve(sizeof(int64_t) * (n_users + 1)));
  COOC_TRY(b_items.reserve(sizeof(int32_t) * (n + 1)));
  if (n_users > 0)
    COOC_HIP_TRY(hipMemcpyAsync(b_user_ptr.p, user_ptr, sizeof(int64_t) * (n_users + 1), hipMemcpyHostToDevice, stream));
  if (n > 0) COOC_HIP_TRY(hipMemcpyAsync(b_items.p, items, sizeof(int32_t) * n, hipMemcpyHostToDevice, stream));
  cooc_device_result r;
  COOC_TRY(count_device(n_users, b_user_ptr.as<int64_t>(), b_items.as<int32_t>(), n, stream, &r));
  std::vector<int32_t> nnz_rows(cfg.n_items);
  COOC_HIP_TRY(hipMemcpy(nnz_rows.data(), r.row_nnz, sizeof(int32_t) * cfg.n_items, hipMemcpyDeviceToHost));
  std::memset(info, 0, sizeof(*info));
  info->nnz = r.nnz;
  info->observed = r.observed;
  info->n_rows = int32_t(std::count_if(nnz_rows.begin(), nnz_rows.end(), [](int32_t x) { return x > 0; }));
  return Status::Ok();
}

Status cooc_ctx::count_owned_host(int64_t n_users, const int64_t *user_ptr, const int32_t *items, cooc_owned_info *info,
                                  cooc_window_info *winfo) {
  COOC_HIP_TRY(hipSetDevice(device));
  if (user_ptr && n_users > 0 && user_ptr[0] != 0) return Status{COOC_ERR_ARG, "user_ptr[0] must be 0"};
  for (int64_t u = 0; u < n_users; u++)
    if (user_ptr[u + 1] < user_ptr[u]) return Status{COOC_ERR_ARG, "user_ptr must be non-decreasing"};
  const int64_t n = n_users > 0 ? user_ptr[n_users] : 0;
  if (n > 0 && !items) return Status{COOC_ERR_ARG, "items is NULL"};
  COOC_TRY(b_user_ptr.reserve(sizeof(int64_t) * (n_users + 1)));
  COOC_TRY(b_items.reserve(sizeof(int32_t) * (n + 1)));
  if (n_users > 0)
    COOC_HIP_TRY(hipMemcpyAsync(b_user_ptr.p, user_ptr, sizeof(int64_t) * (n_users + 1), hipMemcpyHostToDevice, stream));
  else
    COOC_HIP_TRY(hipMemsetAsync(b_user_ptr.p, 0, sizeof(int64_t), stream));
  if (n > 0) COOC_HIP_TRY(hipMemcpyAsync(b_items.p, items, sizeof(int32_t) * n, hipMemcpyHostToDevice, stream));
  cooc_device_result r;
  COOC_TRY(count_owned(n_users, b_user_ptr.as<int64_t>(), b_items.as<int32_t>(), n, stream, info, &r));
  if (winfo) {
    std::vector<int32_t> nnz_rows(cfg.n_items);
    COOC_HIP_TRY(hipMemcpy(nnz_rows.data(), r.row_nnz, sizeof(int32_t) * cfg.n_items, hipMemcpyDeviceToHost));
    std::memset(winfo, 0, sizeof(*winfo));
    winfo->nnz = r.nnz;
    winfo->observed = r.observed;
    winfo->n_rows = int32_t(std::count_if(nnz_rows.begin(), nnz_rows.end(), [](int32_t x) { return x > 0; }));
  }
  return Status::Ok();
}

Status cooc_ctx::copy_batch(int64_t *row_ptr, int32_t *cols, uint32_t *cnt, int16_t *cnt16, int64_t *rowsum,
                            int32_t *rowsum32) {
  if (!have_batch) return Status{COOC_ERR_STATE, "no batch result on this context"};
  COOC_HIP_TRY(hipSetDevice(device));
  const int32_t M = cfg.n_items;
  int64_t *d_rp;
  int32_t *d_col;
  uint32_t *d_cnt;
  COOC_TRY(counter.pack(stream, &d_rp, &d_col, &d_cnt));
  COOC_HIP_TRY(hipStreamSynchronize(stream));
  // the device rows need sorting on the way out when they are not in id order: a relabel's column order, or
  // no order at all (COOC_FLAG_ANY_ORDER)
  const bool resort = batch_result.rank_of || batch_result.unordered;
  if (!resort) {
    if (row_ptr) COOC_HIP_TRY(hipMemcpy(row_ptr, d_rp, sizeof(int64_t) * (M + 1), hipMemcpyDeviceToHost));
    if (cols && batch_nnz) COOC_HIP_TRY(hipMemcpy(cols, d_col, sizeof(int32_t) * batch_nnz, hipMemcpyDeviceToHost));
  }
  if ((cnt || cnt16 || resort) && batch_nnz) {
    std::vector<uint32_t> tmp;
    uint32_t *dst = cnt;
    if (!dst) {
      tmp.resize(batch_nnz);
      dst = tmp.data();
    }
    COOC_HIP_TRY(hipMemcpy(dst, d_cnt, sizeof(uint32_t) * batch_nnz, hipMemcpyDeviceToHost));
    if (resort) {
      // the packed host copy is in ascending column order, each row sorted as (column, count) pairs
      std::vector<int64_t> rp(static_cast<size_t>(M) + 1);
      std::vector<int32_t> cc(static_cast<size_t>(batch_nnz));
      COOC_HIP_TRY(hipMemcpy(rp.data(), d_rp, sizeof(int64_t) * (M + 1), hipMemcpyDeviceToHost));
      COOC_HIP_TRY(hipMemcpy(cc.data(), d_col, sizeof(int32_t) * batch_nnz, hipMemcpyDeviceToHost));
      std::vector<uint64_t> kv;
      for (int32_t a = 0; a < M; a++) {
        const int64_t b0 = rp[size_t(a)], b1 = rp[size_t(a) + 1];
        kv.resize(size_t(b1 - b0));
        for (int64_t i = b0; i < b1; i++) kv[size_t(i - b0)] = (uint64_t(uint32_t(cc[size_t(i)])) << 32) | dst[i];
        std::sort(kv.begin(), kv.end());
        for (int64_t i = b0; i < b1; i++) {
          cc[size_t(i)] = int32_t(kv[size_t(i - b0)] >> 32);
          dst[i] = uint32_t(kv[size_t(i - b0)]);
        }
      }
      if (row_ptr) std::copy(rp.begin(), rp.end(), row_ptr);
      if (cols) std::copy(cc.begin(), cc.end(), cols);
    }
    if (cnt16)  // Int2ShortOpenHashMap value: the count modulo 2^16 as a signed short
      for (int64_t i = 0; i < batch_nnz; i++) cnt16[i] = int16_t(uint16_t(dst[i]));
  } else if (resort && row_ptr) {
    COOC_HIP_TRY(hipMemcpy(row_ptr, d_rp, sizeof(int64_t) * (M + 1), hipMemcpyDeviceToHost));
  }
  if (rowsum || rowsum32) {
    std::vector<int64_t> tmp(M);
    COOC_HIP_TRY(hipMemcpy(tmp.data(), counter.last_rowsum(), sizeof(int64_t) * M, hipMemcpyDeviceToHost));
    if (rowsum) std::memcpy(rowsum, tmp.data(), sizeof(int64_t) * M);
    if (rowsum32)  // Java int accumulation (RowSumAggregator.java:25-27, Int2IntOpenHashMap.addTo)
      for (int32_t a = 0; a < M; a++) rowsum32[a] = int32_t(uint32_t(uint64_t(tmp[a])));
  }
  return Status::Ok();
}

Status cooc_ctx::copy_batch_range(int32_t r0, int32_t r1, int64_t cap, int32_t *cols, uint32_t *cnt, int16_t *cnt16) {
  if (!have_batch) return Status{COOC_ERR_STATE, "no batch result on this context"};
  const int32_t M = cfg.n_items;
  if (r0 < 0 || r1 > M || r0 > r1) return Status{COOC_ERR_ARG, "bad row range"};
  COOC_HIP_TRY(hipSetDevice(device));
  if (!batch_packed) {
    COOC_TRY(counter.pack(stream, &batch_pk_rp, &batch_pk_col, &batch_pk_cnt));
    batch_rp_host.resize(size_t(M) + 1);
    COOC_HIP_TRY(hipMemcpyAsync(batch_rp_host.data(), batch_pk_rp, sizeof(int64_t) * (size_t(M) + 1), hipMemcpyDeviceToHost,
                                stream));
    COOC_HIP_TRY(hipStreamSynchronize(stream));
    batch_packed = true;
  }
  const int64_t e0 = batch_rp_host[size_t(r0)], e1 = batch_rp_host[size_t(r1)], n = e1 - e0;
  if (n > cap) return Status{COOC_ERR_ARG, "rows [" + std::to_string(r0) + ", " + std::to_string(r1) + ") hold " +
                                               std::to_string(n) + " entries, more than " + std::to_string(cap)};
  if (n == 0 || (!cols && !cnt && !cnt16)) return Status::Ok();
  std::vector<int32_t> cc(static_cast<size_t>(n));
  std::vector<uint32_t> vv(static_cast<size_t>(n));
  COOC_HIP_TRY(hipMemcpy(cc.data(), batch_pk_col + e0, sizeof(int32_t) * size_t(n), hipMemcpyDeviceToHost));
  COOC_HIP_TRY(hipMemcpy(vv.data(), batch_pk_cnt + e0, sizeof(uint32_t) * size_t(n), hipMemcpyDeviceToHost));
  if (batch_result.rank_of || batch_result.unordered) {  // ascending column order, as cooc_copy_batch
    std::vector<uint64_t> kv;
    for (int32_t a = r0; a < r1; a++) {
      const int64_t b0 = batch_rp_host[size_t(a)] - e0, b1 = batch_rp_host[size_t(a) + 1] - e0;
      kv.resize(size_t(b1 - b0));
      for (int64_t i = b0; i < b1; i++) kv[size_t(i - b0)] = (uint64_t(uint32_t(cc[size_t(i)])) << 32) | vv[size_t(i)];
      std::sort(kv.begin(), kv.end());
      for (int64_t i = b0; i < b1; i++) {
        cc[size_t(i)] = int32_t(kv[size_t(i - b0)] >> 32);
        vv[size_t(i)] = uint32_t(kv[size_t(i - b0)]);
      }
    }
  }
  if (cols) std::copy(cc.begin(), cc.end(), cols);
  if (cnt) std::copy(vv.begin(), vv.end(), cnt);
  if (cnt16)  // Int2ShortOpenHashMap value: the count modulo 2^16 as a signed short
    for (int64_t i = 0; i < n; i++) cnt16[i] = int16_t(uint16_t(vv[size_t(i)]));
  return Status::Ok();
}

Status cooc_ctx::copy_topk_batch_range(int32_t r0, int32_t r1, int32_t topk, int32_t *sizes, int32_t *values,
                                       double *scores) {
  if (batch_topk <= 0) return Status{COOC_ERR_STATE, "cooc_topk_batch has not run"};
  if (topk != batch_topk)  // the caller's buffers hold topk entries per row
    return Status{COOC_ERR_ARG, "topk " + std::to_string(topk) + " != the scored top-k " + std::to_string(batch_topk)};
  const int32_t M = cfg.n_items;
  if (r0 < 0 || r1 > M || r0 > r1) return Status{COOC_ERR_ARG, "bad row range"};
  COOC_HIP_TRY(hipSetDevice(device));
  const size_t n = size_t(r1 - r0), k = size_t(batch_topk);
  if (sizes && n) COOC_HIP_TRY(hipMemcpy(sizes, b_tk_size.as<int32_t>() + r0, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
  if (values && n)
    COOC_HIP_TRY(hipMemcpy(values, b_tk_val.as<int32_t>() + size_t(r0) * k, sizeof(int32_t) * n * k, hipMemcpyDeviceToHost));
  if (scores && n)
    COOC_HIP_TRY(hipMemcpy(scores, b_tk_score.as<double>() + size_t(r0) * k, sizeof(double) * n * k, hipMemcpyDeviceToHost));
  return Status::Ok();
}

Status cooc_ctx::topk_owned_host(int32_t topk, int32_t flags) {
  if (topk <= 0) return Status{COOC_ERR_ARG, std::to_string(topk) + " is <= 0"};  // ItemRowRescorer...java:52-54
  COOC_HIP_TRY(hipSetDevice(device));
  const int32_t M = cfg.n_items;
  COOC_TRY(b_tk_size.reserve(sizeof(int32_t) * M));
  COOC_TRY(b_tk_val.reserve(sizeof(int32_t) * size_t(M) * topk));
  COOC_TRY(b_tk_score.reserve(sizeof(double) * size_t(M) * topk));
  COOC_TRY(topk_owned(topk, flags, b_tk_size.as<int32_t>(), b_tk_val.as<int32_t>(), b_tk_score.as<double>(), nullptr,
                      stream));
  COOC_HIP_TRY(hipStreamSynchronize(stream));
  batch_topk = topk;
  batch_topk_flags = flags & COOC_FLAG_EXACT_SCORES;
  return Status::Ok();
}

Status cooc_ctx::comm_allgather_i64(int64_t value, int64_t *out) {
  if (!comm) return Status{COOC_ERR_STATE, "cooc_comm_allgather_i64 needs a communicator (cooc_comm_init)"};
  COOC_HIP_TRY(hipSetDevice(device));
  const int32_t W = comm->world();
  COOC_TRY(own_obs.reserve(sizeof(int64_t) * size_t(W + 1)));
  int64_t *d = own_obs.as<int64_t>();
  COOC_HIP_TRY(hipMemcpyAsync(d, &value, sizeof(int64_t), hipMemcpyHostToDevice, stream));
  COOC_TRY(comm->allgather(d, d + 1, sizeof(int64_t), stream));
  COOC_HIP_TRY(hipMemcpyAsync(out, d + 1, sizeof(int64_t) * size_t(W), hipMemcpyDeviceToHost, stream));
  COOC_HIP_TRY(hipStreamSynchronize(stream));
  return Status::Ok();
}

Status cooc_ctx::topk_batch(int32_t topk, int32_t flags, hipStream_t s) {
  if (!have_batch) return Status{COOC_ERR_STATE, "no batch result on this context"};
  if (topk <= 0) return Status{COOC_ERR_ARG, std::to_string(topk) + " is <= 0"};  // ItemRowRescorer...java:52-54
  COOC_HIP_TRY(hipSetDevice(device));
  const int32_t M = cfg.n_items;
  COOC_TRY(b_tk_size.reserve(sizeof(int32_t) * M));
  COOC_TRY(b_tk_val.reserve(sizeof(int32_t) * size_t(M) * topk));
  COOC_TRY(b_tk_score.reserve(sizeof(double) * size_t(M) * topk));
  COOC_TRY(topk_batch_device(topk, flags, nullptr, b_tk_size.as<int32_t>(), b_tk_val.as<int32_t>(),
                             b_tk_score.as<double>(), s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  batch_topk = topk;
  batch_topk_flags = flags & COOC_FLAG_EXACT_SCORES;
  return Status::Ok();
}

Status cooc_ctx::topk_batch_device(int32_t topk, int32_t flags, const int64_t *d_rowsum_global, int32_t *d_sizes,
                                   int32_t *d_values, double *d_scores, hipStream_t s) {
  if (!have_batch) return Status{COOC_ERR_STATE, "no batch result on this context"};
  if (topk <= 0) return Status{COOC_ERR_ARG, std::to_string(topk) + " is <= 0"};  // ItemRowRescorer...java:52-54
  COOC_HIP_TRY(hipSetDevice(device));
  const int32_t M = cfg.n_items;
  COOC_TRY(b_obs3.reserve(sizeof(int64_t) * 4));
  // (the batch is complete: cooc_count_device* returned after draining its stream)
  const cooc::CountResult &r = batch_result;
  return cooc::launch_rescore_batch(s, M, r.row_base, r.row_nnz, r.col, r.cnt, r.dense,
                                    d_rowsum_global ? d_rowsum_global : r.rowsum, (flags & COOC_FLAG_EXACT_SCORES) != 0,
                                    topk, b_obs3.as<int64_t>(), b_llr_terms, d_sizes, d_values, d_scores, r.rank_of,
                                    r.unordered, r.nnz, d_rowsum_global != nullptr);
}

Status cooc_ctx::llr(int64_t n, const int64_t *k, double *out) {
  if (n == 0) return Status::Ok();
  COOC_HIP_TRY(hipSetDevice(device));
  cooc::DevBuf dk, dout;
  Status st = [&]() -> Status {
    COOC_TRY(dk.reserve(sizeof(int64_t) * 4 * size_t(n)));
    COOC_TRY(dout.reserve(sizeof(double) * size_t(n)));
    COOC_HIP_TRY(hipMemcpyAsync(dk.p, k, sizeof(int64_t) * 4 * size_t(n), hipMemcpyHostToDevice, stream));
    COOC_TRY(cooc::launch_llr(stream, n, dk.as<int64_t>(), dout.as<double>()));
    COOC_HIP_TRY(hipMemcpyAsync(out, dout.p, sizeof(double) * size_t(n), hipMemcpyDeviceToHost, stream));
    COOC_HIP_TRY(hipStreamSynchronize(stream));
    return Status::Ok();
  }();
  dk.release();
  dout.release();
  return st;
}

Status cooc_ctx::topk_items(int32_t k, int32_t flags, int32_t n, const int32_t *items, int32_t *sizes,
                            int32_t *values, double *scores) {
  if (!have_batch) return Status{COOC_ERR_STATE, "no batch result on this context"};
  const int32_t M = cfg.n_items;
  for (int32_t i = 0; i < n; i++)
    if (items[i] < 0 || items[i] >= M) return Status{COOC_ERR_ARG, std::to_string(items[i]) + " is not an item"};
  if (batch_topk != k || batch_topk_flags != (flags & COOC_FLAG_EXACT_SCORES)) COOC_TRY(topk_batch(k, flags, stream));
  COOC_HIP_TRY(hipSetDevice(device));
  const size_t kk = size_t(k);
  for (int32_t i = 0; i < n; i++) {
    const size_t a = size_t(items[i]);
    COOC_HIP_TRY(hipMemcpy(sizes + i, b_tk_size.as<int32_t>() + a, sizeof(int32_t), hipMemcpyDeviceToHost));
    COOC_HIP_TRY(hipMemcpy(values + i * kk, b_tk_val.as<int32_t>() + a * kk, sizeof(int32_t) * kk, hipMemcpyDeviceToHost));
    COOC_HIP_TRY(hipMemcpy(scores + i * kk, b_tk_score.as<double>() + a * kk, sizeof(double) * kk, hipMemcpyDeviceToHost));
  }
  return Status::Ok();
}

Status cooc_ctx::copy_topk_batch(int32_t *sizes, int32_t *values, double *scores) {
  if (batch_topk <= 0) return Status{COOC_ERR_STATE, "cooc_topk_batch has not run"};
  COOC_HIP_TRY(hipSetDevice(device));
  const size_t M = size_t(cfg.n_items), k = size_t(batch_topk);
  if (sizes) COOC_HIP_TRY(hipMemcpy(sizes, b_tk_size.p, sizeof(int32_t) * M, hipMemcpyDeviceToHost));
  if (values) COOC_HIP_TRY(hipMemcpy(values, b_tk_val.p, sizeof(int32_t) * M * k, hipMemcpyDeviceToHost));
  if (scores) COOC_HIP_TRY(hipMemcpy(scores, b_tk_score.p, sizeof(double) * M * k, hipMemcpyDeviceToHost));
  return Status::Ok();
}

Status cooc_ctx::verify_batch(int32_t flags, uint64_t *d_row_checksum, int64_t *out8, hipStream_t s) {
  if (!have_batch) return Status{COOC_ERR_STATE, "no batch result on this context"};
  const bool sym = (flags & COOC_VERIFY_SYMMETRY) != 0;
  if (sym && batch_owned)
    return Status{COOC_ERR_ARG, "COOC_VERIFY_SYMMETRY needs a whole result (not one part's owned rows)"};
  COOC_HIP_TRY(hipSetDevice(device));
  COOC_TRY(b_verify.reserve(sizeof(uint64_t) * 8));
  // (the batch is complete: cooc_count_device* returned after draining its stream)
  COOC_TRY(cooc::launch_verify(s, cfg.n_items, batch_result, sym && !batch_result.dense, d_row_checksum,
                               b_verify.as<unsigned long long>()));
  uint64_t h[8];
  COOC_HIP_TRY(hipMemcpyAsync(h, b_verify.p, sizeof(h), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  for (int i = 0; i < 8; i++) out8[i] = int64_t(h[i]);
  if (!sym || batch_result.dense || batch_result.unordered) out8[5] = -1;
  out8[6] = out8[7] = 0;
  return Status::Ok();
}
