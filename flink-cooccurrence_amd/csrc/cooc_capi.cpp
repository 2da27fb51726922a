// cooc_capi.cpp — the C-ABI of include/cooc.h over the HIP pipeline (cooc_count.hip) and the
// resident streaming state (cooc_stream.cpp).  Error behaviour mirrors the reference: argument
// errors (IllegalArgumentException, e.g. ItemRowRescorer...java:52-54) -> COOC_ERR_ARG, state
// errors (IllegalStateException, e.g. ItemRowRescorer...java:72-79,91-93) -> COOC_ERR_STATE.
#include "cooc_ctx.h"

#include <cstring>
#include <exception>
#include <new>
#include <vector>

using cooc::Status;

namespace cooc {
Status selftest_scan(const void *d_in, void *d_out, int64_t n, int32_t flags, hipStream_t s, int64_t *h_err);  // cooc_verify.hip
Status selftest_radix(const void *kin, const void *vin, void *kout, void *vout, int64_t n, int32_t key_bytes,
                      int32_t bit0, int32_t bit1, int32_t desc, hipStream_t s);  // cooc_verify.hip
Status selftest_select(const uint8_t *flag, int64_t n, int32_t *out, int32_t *n_sel, hipStream_t s);
}

namespace {

int fail(cooc_ctx *ctx, const Status &s) {
  if (ctx)
    ctx->last_error = s.msg;
  else
    cooc_ctx::create_error() = s.msg;  // no context: cooc_last_error(NULL)
  return s.code;
}

int fail(cooc_ctx *ctx, int code, const std::string &msg) { return fail(ctx, Status{code, msg}); }

// Exception firewall: no C++ exception crosses the C-ABI (a JVM caller cannot unwind it).
// std::bad_alloc -> COOC_ERR_OOM, anything else -> COOC_ERR_STATE, with the message kept.
template <class F>
int guarded(cooc_ctx *ctx, F &&f) {
  try {
    return f();
  } catch (const std::bad_alloc &) {
    return fail(ctx, COOC_ERR_OOM, "host allocation failed (std::bad_alloc)");
  } catch (const std::exception &e) {
    return fail(ctx, COOC_ERR_STATE, std::string("internal error: ") + e.what());
  } catch (...) {
    return fail(ctx, COOC_ERR_STATE, "internal error (unknown exception)");
  }
}

}  // namespace

extern "C" {

int cooc_abi_version(void) { return COOC_ABI_VERSION; }

const char *cooc_status_string(int status) {
  switch (status) {
    case COOC_OK: return "ok";
    case COOC_ERR_ARG: return "invalid argument";
    case COOC_ERR_STATE: return "invalid state";
    case COOC_ERR_HIP: return "HIP runtime error";
    case COOC_ERR_OOM: return "device out of memory";
    case COOC_ERR_OVERFLOW: return "uint32 count overflow";
    default: return "unknown status";
  }
}

int cooc_create(const cooc_config *cfg, cooc_ctx **out) {
  return guarded(nullptr, [&]() -> int {
    if (!cfg || !out) return COOC_ERR_ARG;
    *out = nullptr;
    auto ctx = std::make_unique<cooc_ctx>();
    Status s = ctx->init(*cfg);
    if (!s.ok()) {
      // no context to carry the message: keep it in a thread-local for cooc_last_error(NULL)
      cooc_ctx::create_error() = s.msg;
      return s.code;
    }
    *out = ctx.release();
    return COOC_OK;
  });
}

int cooc_create_on(const cooc_config *cfg, const int32_t *devices, int32_t n_devices, int32_t subtask,
                   cooc_ctx **out) {
  return guarded(nullptr, [&]() -> int {
    if (!cfg || !out || !devices || n_devices <= 0 || subtask < 0) {
      cooc_ctx::create_error() = "cooc_create_on: bad devices / subtask arguments";
      return COOC_ERR_ARG;
    }
    int n_dev = 0;
    if (hipGetDeviceCount(&n_dev) != hipSuccess) n_dev = 0;
    for (int32_t i = 0; i < n_devices; i++)
      if (devices[i] < 0 || devices[i] >= n_dev) {
        cooc_ctx::create_error() = "device " + std::to_string(devices[i]) + " is not in [0, " + std::to_string(n_dev) + ")";
        return COOC_ERR_ARG;
      }
    cooc_config c = *cfg;
    c.device = devices[subtask % n_devices];
    return cooc_create(&c, out);
  });
}

void cooc_destroy(cooc_ctx *ctx) { delete ctx; }

const char *cooc_last_error(const cooc_ctx *ctx) {
  return ctx ? ctx->last_error.c_str() : cooc_ctx::create_error().c_str();
}

int cooc_count_device(cooc_ctx *ctx, int64_t n_users, const int64_t *d_user_ptr, const int32_t *d_items,
                      int64_t n_interactions, void *hip_stream, cooc_device_result *out) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !out) return COOC_ERR_ARG;
    if (n_users < 0 || n_interactions < 0 || (n_users > 0 && (!d_user_ptr || (n_interactions > 0 && !d_items))))
      return fail(ctx, COOC_ERR_ARG, "bad CSR arguments");
    Status s = ctx->count_device(n_users, d_user_ptr, d_items, n_interactions,
                                 static_cast<hipStream_t>(hip_stream), out);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_count_device_owned(cooc_ctx *ctx, int64_t n_users, const int64_t *d_user_ptr, const int32_t *d_items,
                            int64_t n_interactions, const int32_t *d_owner, int32_t part,
                            const int64_t *d_item_counts, int64_t n_total, void *hip_stream, cooc_device_result *out) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !out) return COOC_ERR_ARG;
    if (n_users < 0 || n_interactions < 0 || (n_users > 0 && (!d_user_ptr || (n_interactions > 0 && !d_items))))
      return fail(ctx, COOC_ERR_ARG, "bad CSR arguments");
    if (!d_owner || !d_item_counts || n_total < 0) return fail(ctx, COOC_ERR_ARG, "bad ownership arguments");
    Status s = ctx->count_device_owned(n_users, d_user_ptr, d_items, n_interactions, d_owner, part, d_item_counts,
                                       n_total, static_cast<hipStream_t>(hip_stream), out);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_item_counts(cooc_ctx *ctx, const int32_t *d_items, int64_t n_interactions, int64_t *d_counts, void *hip_stream) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !d_counts || n_interactions < 0 || (n_interactions > 0 && !d_items))
      return fail(ctx, COOC_ERR_ARG, "bad item_counts arguments");
    (void)hipSetDevice(ctx->device);
    Status s = cooc::launch_item_counts(static_cast<hipStream_t>(hip_stream), d_items, n_interactions, ctx->cfg.n_items,
                                        d_counts);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_copy_column_order(cooc_ctx *ctx, int32_t *rank_of) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !rank_of) return COOC_ERR_ARG;
    if (!ctx->have_batch) return fail(ctx, COOC_ERR_STATE, "no batch result on this context");
    (void)hipSetDevice(ctx->device);
    const int32_t M = ctx->cfg.n_items;
    if (!ctx->batch_result.rank_of) {
      for (int32_t a = 0; a < M; a++) rank_of[a] = a;
      return COOC_OK;
    }
    hipError_t e = hipMemcpy(rank_of, ctx->batch_result.rank_of, sizeof(int32_t) * size_t(M), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return fail(ctx, COOC_ERR_HIP, std::string("hipMemcpy: ") + hipGetErrorString(e));
    return COOC_OK;
  });
}

int cooc_count_host(cooc_ctx *ctx, int64_t n_users, const int64_t *user_ptr, const int32_t *items,
                    cooc_window_info *info) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !info) return COOC_ERR_ARG;
    if (n_users < 0 || (n_users > 0 && !user_ptr)) return fail(ctx, COOC_ERR_ARG, "bad CSR arguments");
    Status s = ctx->count_host(n_users, user_ptr, items, info);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_copy_batch(cooc_ctx *ctx, int64_t *row_ptr, int32_t *cols, uint32_t *cnt, int16_t *cnt16, int64_t *rowsum,
                    int32_t *rowsum32) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    Status s = ctx->copy_batch(row_ptr, cols, cnt, cnt16, rowsum, rowsum32);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_copy_batch_range(cooc_ctx *ctx, int32_t row_begin, int32_t row_end, int64_t cap, int32_t *cols, uint32_t *cnt,
                          int16_t *cnt16) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    Status s = ctx->copy_batch_range(row_begin, row_end, cap, cols, cnt, cnt16);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_copy_topk_batch_range(cooc_ctx *ctx, int32_t row_begin, int32_t row_end, int32_t topk, int32_t *sizes,
                               int32_t *values, double *scores) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    Status s = ctx->copy_topk_batch_range(row_begin, row_end, topk, sizes, values, scores);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_topk_owned_host(cooc_ctx *ctx, int32_t topk, int32_t flags) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    Status s = ctx->topk_owned_host(topk, flags);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_comm_allgather_i64(cooc_ctx *ctx, int64_t value, int64_t *out) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !out) return COOC_ERR_ARG;
    Status s = ctx->comm_allgather_i64(value, out);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_topk_batch(cooc_ctx *ctx, int32_t topk, int32_t flags, void *hip_stream) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    // NULL: the context's own stream (the count it scores has already drained; see cooc.h)
    Status s = ctx->topk_batch(topk, flags, hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->stream);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_topk_batch_device(cooc_ctx *ctx, int32_t topk, int32_t flags, const int64_t *d_rowsum_global,
                           int32_t *d_sizes, int32_t *d_values, double *d_scores, void *hip_stream) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    if (!d_sizes || !d_values || !d_scores) return fail(ctx, COOC_ERR_ARG, "bad topk output buffers");
    Status s = ctx->topk_batch_device(topk, flags, d_rowsum_global, d_sizes, d_values, d_scores,
                                      static_cast<hipStream_t>(hip_stream));
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_copy_topk_batch(cooc_ctx *ctx, int32_t *sizes, int32_t *values, double *scores) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    Status s = ctx->copy_topk_batch(sizes, values, scores);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_llr(cooc_ctx *ctx, int64_t n, const int64_t *k, double *out) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    if (n < 0 || (n > 0 && (!k || !out))) return fail(ctx, COOC_ERR_ARG, "bad llr arguments");
    Status s = ctx->llr(n, k, out);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_topk_items(cooc_ctx *ctx, int32_t k, int32_t flags, int32_t n, const int32_t *items, int32_t *out_sizes,
                    int32_t *out_items, double *out_scores) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    if (n < 0 || (n > 0 && (!items || !out_sizes || !out_items || !out_scores)))
      return fail(ctx, COOC_ERR_ARG, "bad topk_items arguments");
    Status s = ctx->topk_items(k, flags, n, items, out_sizes, out_items, out_scores);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_submit_batch(cooc_ctx *ctx, int64_t window_ts, int32_t n_users, const int32_t *user_ids,
                      const int64_t *user_ptr, const int32_t *items) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    if (n_users < 0 || (n_users > 0 && (!user_ids || !user_ptr))) return fail(ctx, COOC_ERR_ARG, "bad batch arguments");
    Status s = ctx->stream_state.submit(*ctx, window_ts, n_users, user_ids, user_ptr, items);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_finish_window(cooc_ctx *ctx, int64_t window_ts, cooc_window_info *info) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !info) return COOC_ERR_ARG;
    Status s = ctx->stream_state.finish(*ctx, window_ts, info);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_copy_window_delta(cooc_ctx *ctx, int32_t *rows, int64_t *row_ptr, int32_t *cols, uint32_t *cnt,
                           int16_t *cnt16) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    Status s = ctx->stream_state.copy_delta(*ctx, rows, row_ptr, cols, cnt, cnt16);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_copy_window_delta_range(cooc_ctx *ctx, int32_t row_begin, int32_t row_end, int64_t cap, int32_t *cols, uint32_t *cnt,
                                 int16_t *cnt16) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    Status s = ctx->stream_state.copy_delta_range(*ctx, row_begin, row_end, cap, cols, cnt, cnt16);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_copy_window_rowsums(cooc_ctx *ctx, int32_t *items, int64_t *delta, int32_t *delta32) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    Status s = ctx->stream_state.copy_rowsums(*ctx, items, delta, delta32);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_copy_window_topk(cooc_ctx *ctx, int32_t *rows, int32_t *sizes, int32_t *values, double *scores) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    Status s = ctx->stream_state.copy_topk(*ctx, rows, sizes, values, scores);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_global_rowsums(cooc_ctx *ctx, int64_t *exact, int32_t *v32) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    Status s = ctx->stream_state.global_rowsums(*ctx, exact, v32);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_global_observed(cooc_ctx *ctx, int64_t *exact, int64_t *rescorer) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    if (exact) *exact = ctx->stream_state.observed_exact;
    if (rescorer) *rescorer = ctx->stream_state.observed_ref;
    return COOC_OK;
  });
}

int cooc_global_row_nnz(cooc_ctx *ctx, int32_t item, int64_t *nnz) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !nnz) return COOC_ERR_ARG;
    Status s = ctx->stream_state.global_row_nnz(*ctx, item, nnz);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_global_row(cooc_ctx *ctx, int32_t item, int32_t *cols, uint32_t *cnt, int16_t *cnt16) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    Status s = ctx->stream_state.global_row(*ctx, item, cols, cnt, cnt16);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_op_process_elements(cooc_ctx *ctx, int64_t n, const int32_t *users, const int32_t *items,
                             const int64_t *ts, int64_t *n_late) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    if (n < 0 || (n > 0 && (!users || !items || !ts))) return fail(ctx, COOC_ERR_ARG, "bad element arrays");
    Status s = ctx->op.process_elements(*ctx, n, users, items, ts, n_late);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_op_process_watermark(cooc_ctx *ctx, int64_t watermark, int32_t *fired, cooc_window_info *info) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !fired || !info) return COOC_ERR_ARG;
    Status s = ctx->op.process_watermark(*ctx, watermark, fired, info);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_op_counters(cooc_ctx *ctx, int64_t *counters5) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !counters5) return COOC_ERR_ARG;
    counters5[0] = ctx->op.late_elements;
    counters5[1] = ctx->stream_state.observed_exact;
    counters5[2] = ctx->stream_state.rowsum_acc;
    counters5[3] = ctx->stream_state.rescored_items;
    counters5[4] = ctx->stream_state.observed_ref;
    return COOC_OK;
  });
}

// Device-pointer entry points run on the caller's stream; NULL is the HIP null stream, which orders
// them with hipMemcpy and with torch's default stream (cooc.h, stream contract).
static hipStream_t stream_of(cooc_ctx *, void *s) { return static_cast<hipStream_t>(s); }

int cooc_partition_plan(cooc_ctx *ctx, int32_t n_parts, int64_t *h_entries) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !h_entries) return COOC_ERR_ARG;
    if (!ctx->have_batch) return fail(ctx, COOC_ERR_STATE, "no cooc_count_device result to partition");
    if (ctx->batch_result.unordered)
      return fail(ctx, COOC_ERR_STATE, "a COOC_FLAG_ANY_ORDER result cannot be partitioned (the merge needs ordered rows)");
    Status s = hipSetDevice(ctx->device) == hipSuccess
                   ? ctx->sharder.plan(ctx->batch_result, ctx->cfg.n_items, n_parts, ctx->stream, h_entries)
                   : Status{COOC_ERR_HIP, "hipSetDevice"};
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_partition_pack(cooc_ctx *ctx, int32_t n_parts, int32_t *d_row_nnz, uint64_t *d_entries, void *hip_stream) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    if (!ctx->have_batch) return fail(ctx, COOC_ERR_STATE, "no cooc_count_device result to partition");
    (void)hipSetDevice(ctx->device);
    hipStream_t s = stream_of(ctx, hip_stream);
    Status st = ctx->sharder.pack(ctx->batch_result, ctx->cfg.n_items, n_parts, s, d_row_nnz, d_entries);
    return st.ok() ? COOC_OK : fail(ctx, st);
  });
}

int cooc_copy_rowsum_device(cooc_ctx *ctx, int64_t *d_rowsum, void *hip_stream) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !d_rowsum) return COOC_ERR_ARG;
    if (!ctx->have_batch) return fail(ctx, COOC_ERR_STATE, "no cooc_count_device result");
    (void)hipSetDevice(ctx->device);
    hipError_t e = hipMemcpyAsync(d_rowsum, ctx->batch_result.rowsum, sizeof(int64_t) * ctx->cfg.n_items,
                                  hipMemcpyDeviceToDevice, stream_of(ctx, hip_stream));
    if (e != hipSuccess) return fail(ctx, COOC_ERR_HIP, std::string("hipMemcpyAsync: ") + hipGetErrorString(e));
    return COOC_OK;
  });
}

int cooc_merge_partitions(cooc_ctx *ctx, int32_t n_parts, int32_t part, const int32_t *d_recv_row_nnz,
                          const uint64_t *d_recv_entries, const int64_t *d_rowsum_global, void *hip_stream,
                          cooc_device_result *out) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !out || !d_recv_row_nnz) return COOC_ERR_ARG;
    if (n_parts < 1) return fail(ctx, COOC_ERR_ARG, "n_parts must be >= 1");
    (void)hipSetDevice(ctx->device);
    cooc::MergeResult m;
    Status s = ctx->sharder.merge(ctx->cfg.n_items, n_parts, part, d_recv_row_nnz, d_recv_entries, d_rowsum_global,
                                  stream_of(ctx, hip_stream), &m);
    if (!s.ok()) return fail(ctx, s);
    out->n_items = m.n_rows;
    out->nnz = -1;
    out->observed = -1;
    out->row_base = m.row_base;
    out->row_nnz = m.row_nnz;
    out->col = m.col;
    out->cnt = m.cnt;
    out->rowsum = m.rowsum;
    out->dense = nullptr;
    return COOC_OK;
  });
}

int cooc_comm_unique_id(uint8_t *id) {
  return guarded(nullptr, [&]() -> int {
    if (!id) return COOC_ERR_ARG;
    Status s = cooc::Comm::unique_id(id);
    return s.ok() ? COOC_OK : fail(nullptr, s);
  });
}

int cooc_comm_init(cooc_ctx *ctx, const uint8_t *id, int32_t rank, int32_t world) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !id) return COOC_ERR_ARG;
    if (world < 1 || rank < 0 || rank >= world) return fail(ctx, COOC_ERR_ARG, "rank must lie in [0, world)");
    if (ctx->comm) return fail(ctx, COOC_ERR_STATE, "the context already has a communicator");
    auto c = std::make_unique<cooc::Comm>();
    Status s = c->init_rccl(id, rank, world, ctx->device);
    if (!s.ok()) return fail(ctx, s);
    ctx->comm = std::move(c);
    return COOC_OK;
  });
}

int cooc_comm_init_ops(cooc_ctx *ctx, int32_t rank, int32_t world, const cooc_comm_ops *ops, void *user) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !ops) return COOC_ERR_ARG;
    if (world < 1 || rank < 0 || rank >= world) return fail(ctx, COOC_ERR_ARG, "rank must lie in [0, world)");
    if (ctx->comm) return fail(ctx, COOC_ERR_STATE, "the context already has a communicator");
    auto c = std::make_unique<cooc::Comm>();
    Status s = c->init_ops(rank, world, *ops, user);
    if (!s.ok()) return fail(ctx, s);
    ctx->comm = std::move(c);
    return COOC_OK;
  });
}

int cooc_count_owned(cooc_ctx *ctx, int64_t n_users, const int64_t *d_user_ptr, const int32_t *d_items,
                     int64_t n_interactions, void *hip_stream, cooc_owned_info *info, cooc_device_result *out) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !out || !info) return COOC_ERR_ARG;
    if (n_users < 0 || n_interactions < 0 || (n_users > 0 && (!d_user_ptr || (n_interactions > 0 && !d_items))))
      return fail(ctx, COOC_ERR_ARG, "bad CSR arguments");
    Status s = ctx->count_owned(n_users, d_user_ptr, d_items, n_interactions, static_cast<hipStream_t>(hip_stream),
                                info, out);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_count_owned_host(cooc_ctx *ctx, int64_t n_users, const int64_t *user_ptr, const int32_t *items,
                          cooc_owned_info *info, cooc_window_info *winfo) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !info) return COOC_ERR_ARG;
    if (n_users < 0 || (n_users > 0 && !user_ptr)) return fail(ctx, COOC_ERR_ARG, "bad CSR arguments");
    Status s = ctx->count_owned_host(n_users, user_ptr, items, info, winfo);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_topk_owned(cooc_ctx *ctx, int32_t topk, int32_t flags, int32_t *d_sizes, int32_t *d_values, double *d_scores,
                    int64_t *d_rowsum_global, void *hip_stream) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    if (!d_sizes || !d_values || !d_scores) return fail(ctx, COOC_ERR_ARG, "bad topk output buffers");
    Status s = ctx->topk_owned(topk, flags, d_sizes, d_values, d_scores, d_rowsum_global,
                               static_cast<hipStream_t>(hip_stream));
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_snake_owner(const int64_t *counts, int32_t n_items, int32_t world, int32_t head, int32_t *owner) {
  return guarded(nullptr, [&]() -> int {
    if (n_items < 0 || world < 1 || head < 0 || (n_items > 0 && (!counts || !owner))) {
      cooc_ctx::create_error() = "cooc_snake_owner: bad arguments";
      return COOC_ERR_ARG;
    }
    cooc::snake_owner_host(counts, n_items, world, head, owner);
    return COOC_OK;
  });
}

int cooc_shard_plan(cooc_ctx *ctx, int64_t n_users, const int64_t *d_user_ptr, const int32_t *d_items,
                    int64_t n_interactions, int32_t n_parts, uint64_t *d_desc, int32_t *d_row_counts,
                    uint16_t *d_arena, int64_t arena_cap, void *hip_stream, int64_t *h_send, int64_t *h_info) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !h_send || !h_info || !d_row_counts || !d_arena) return COOC_ERR_ARG;
    if (n_users < 0 || n_interactions < 0) return fail(ctx, COOC_ERR_ARG, "negative size");
    if (n_interactions > 0 && (!d_user_ptr || !d_items || !d_desc)) return fail(ctx, COOC_ERR_ARG, "NULL input");
    if (n_parts < 1) return fail(ctx, COOC_ERR_ARG, "n_parts must be >= 1");
    (void)hipSetDevice(ctx->device);
    ctx->have_batch = false;
    Status s = ctx->apply_user_cut(n_users, &d_user_ptr, &d_items, &n_interactions, stream_of(ctx, hip_stream));
    if (s.ok())
      s = ctx->counter.shard_plan(n_users, d_user_ptr, d_items, n_interactions, n_parts, stream_of(ctx, hip_stream),
                                  d_desc, d_row_counts, d_arena, arena_cap, h_send, h_info, h_info + 1);
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_shard_count(cooc_ctx *ctx, int32_t n_parts, int32_t part, const int32_t *d_recv_row_counts,
                     const uint64_t *d_recv_desc, int64_t n_recv, const uint16_t *d_arena_all, int64_t arena_stride,
                     void *hip_stream, cooc_device_result *out) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !out || !d_recv_row_counts || !d_arena_all) return COOC_ERR_ARG;
    if (n_recv > 0 && !d_recv_desc) return fail(ctx, COOC_ERR_ARG, "NULL descriptors");
    if (n_parts < 1) return fail(ctx, COOC_ERR_ARG, "n_parts must be >= 1");
    (void)hipSetDevice(ctx->device);
    ctx->have_batch = false;
    hipStream_t s = stream_of(ctx, hip_stream);
    cooc::CountResult r;
    Status st = ctx->counter.shard_count(n_parts, part, d_recv_row_counts, d_recv_desc, n_recv, d_arena_all,
                                         arena_stride, s, &r, ctx->timer.enabled ? &ctx->timer : nullptr);
    if (!st.ok()) return fail(ctx, st);
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) return fail(ctx, COOC_ERR_HIP, std::string("hipStreamSynchronize: ") + hipGetErrorString(e));
    cooc::PlanTotals t;
    st = ctx->counter.read_totals(&t);
    if (!st.ok()) return fail(ctx, st);
    if (t.err & 2) return fail(ctx, COOC_ERR_OVERFLOW, "a co-occurrence count exceeded uint32");
    out->n_items = ctx->counter.last_rows();
    out->nnz = t.nnz_total;
    out->observed = r.observed;
    out->row_base = r.row_base;
    out->row_nnz = r.row_nnz;
    out->col = r.col;
    out->cnt = r.cnt;
    out->rowsum = r.rowsum;
    out->dense = r.dense;
    return COOC_OK;
  });
}

int cooc_verify_batch(cooc_ctx *ctx, int32_t flags, uint64_t *d_row_checksum, int64_t *out8, void *hip_stream) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !out8) return COOC_ERR_ARG;
    if (flags & ~COOC_VERIFY_SYMMETRY) return fail(ctx, COOC_ERR_ARG, "unknown cooc_verify_batch flags");
    Status s = ctx->verify_batch(flags, d_row_checksum, out8, static_cast<hipStream_t>(hip_stream));
    return s.ok() ? COOC_OK : fail(ctx, s);
  });
}

int cooc_selftest_scan(const void *d_in, void *d_out, int64_t n, int32_t flags, int64_t *diag, void *hip_stream) {
  return guarded(nullptr, [&]() -> int {
    if (!d_in || !d_out || n < 0 || (flags & ~15)) return COOC_ERR_ARG;
    int64_t e = 0;
    Status s = cooc::selftest_scan(d_in, d_out, n, flags, static_cast<hipStream_t>(hip_stream), &e);
    if (diag) *diag = e;
    return s.ok() ? COOC_OK : fail(nullptr, s);
  });
}

int cooc_selftest_radix(const void *d_keys_in, const void *d_vals_in, void *d_keys_out, void *d_vals_out, int64_t n,
                        int32_t key_bytes, int32_t bit0, int32_t bit1, int32_t descending, void *hip_stream) {
  return guarded(nullptr, [&]() -> int {
    if (n < 0 || (n > 0 && (!d_keys_in || !d_vals_in || !d_keys_out || !d_vals_out)) ||
        (key_bytes != 4 && key_bytes != 8) || bit0 < 0 || bit1 > 8 * key_bytes || bit0 > bit1)
      return COOC_ERR_ARG;
    Status s = cooc::selftest_radix(d_keys_in, d_vals_in, d_keys_out, d_vals_out, n, key_bytes, bit0, bit1, descending,
                                    static_cast<hipStream_t>(hip_stream));
    return s.ok() ? COOC_OK : fail(nullptr, s);
  });
}

int cooc_selftest_select(const uint8_t *d_flags, int64_t n, int32_t *d_out, int32_t *d_n_sel, void *hip_stream) {
  return guarded(nullptr, [&]() -> int {
    if (n < 0 || !d_n_sel || (n > 0 && (!d_flags || !d_out))) return COOC_ERR_ARG;
    Status s = cooc::selftest_select(d_flags, n, d_out, d_n_sel, static_cast<hipStream_t>(hip_stream));
    return s.ok() ? COOC_OK : fail(nullptr, s);
  });
}

int cooc_set_kernel_timing(cooc_ctx *ctx, int32_t enable) {
  return guarded(ctx, [&]() -> int {
    if (!ctx) return COOC_ERR_ARG;
    ctx->timer.enabled = enable != 0;
    return COOC_OK;
  });
}

int cooc_last_kernel_ms(cooc_ctx *ctx, float *accumulate_ms) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !accumulate_ms) return COOC_ERR_ARG;
    if (!ctx->timer.enabled) return fail(ctx, COOC_ERR_STATE, "kernel timing is off");
    hipError_t e = hipEventElapsedTime(accumulate_ms, ctx->timer.acc_begin, ctx->timer.acc_end);
    if (e != hipSuccess) return fail(ctx, COOC_ERR_HIP, std::string("hipEventElapsedTime: ") + hipGetErrorString(e));
    return COOC_OK;
  });
}

int cooc_last_sort_rows(cooc_ctx *ctx, int64_t *rows, int64_t *pairs) {
  return guarded(ctx, [&]() -> int {
    if (!ctx || !rows || !pairs) return COOC_ERR_ARG;
    *rows = ctx->counter.last_deferred_rows();
    *pairs = ctx->counter.last_deferred_pairs();
    return COOC_OK;
  });
}

}  // extern "C"
