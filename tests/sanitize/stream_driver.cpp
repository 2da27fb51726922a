// The streaming operator's host bookkeeping under AddressSanitizer + UndefinedBehaviorSanitizer: the library's
// host code (cooc_stream.cpp's user slots, history arena, staging, window agreement and copy-out views;
// cooc_ctx.cpp; cooc_capi.cpp's argument checks) compiled with -fsanitize on the host side only
// (scripts/build_asan.sh), the kernels as usual.  Drives the C-ABI operator mirror
// (NonSampledUserInteractionCounterOneInputStreamOperator, NonSampled...java:80-165) over random click logs --
// a small universe (the dense-tile window path) and a large one (the large-universe window path) -- with
// late records, empty windows, every copy-out call (whole, two-phase, in row ranges with exact and short
// caps), the global snapshots and invalid arguments, and checks the invariants that need no oracle: every
// delta row sums to its row-sum update, the row sums add up to the window's observed pairs, the accumulators
// add up.  Any out-of-bounds host access or undefined operation aborts; prints "stream_asan ok".
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "cooc.h"

#define CHECK(c)                                                              \
  do {                                                                        \
    if (!(c)) {                                                               \
      std::fprintf(stderr, "check failed at %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)
#define OK(call)                                                                                       \
  do {                                                                                                 \
    const int rc_ = (call);                                                                            \
    if (rc_ != 0) {                                                                                    \
      std::fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, cooc_last_error(ctx));                 \
      std::exit(1);                                                                                    \
    }                                                                                                  \
  } while (0)

namespace {

int64_t g_windows = 0, g_entries = 0;

// Every output of one fired window, with the invariants.
void read_window(cooc_ctx *ctx, const cooc_window_info &info, int32_t M, int32_t topk) {
  const int32_t n = info.n_rows;
  std::vector<int32_t> rows(n), cols(info.nnz);
  std::vector<int64_t> rp(n + 1), delta(n);
  std::vector<uint32_t> cnt(info.nnz);
  std::vector<int16_t> c16(info.nnz);
  std::vector<int32_t> items(n), d32(n);
  OK(cooc_copy_window_delta(ctx, rows.data(), rp.data(), nullptr, nullptr, nullptr));  // (two-phase: sizes)
  OK(cooc_copy_window_delta(ctx, rows.data(), rp.data(), cols.data(), cnt.data(), c16.data()));
  OK(cooc_copy_window_rowsums(ctx, items.data(), delta.data(), d32.data()));
  CHECK(rp[0] == 0 && rp[n] == info.nnz);
  int64_t total = 0;
  for (int32_t r = 0; r < n; r++) {
    CHECK(rows[r] >= 0 && rows[r] < M && (r == 0 || rows[r] > rows[r - 1]));
    CHECK(items[r] == rows[r]);
    int64_t s = 0;
    for (int64_t e = rp[r]; e < rp[r + 1]; e++) {
      CHECK(cols[e] >= 0 && cols[e] < M && cnt[e] > 0 && (e == rp[r] || cols[e] > cols[e - 1]));
      CHECK(c16[e] == int16_t(uint16_t(cnt[e])));
      s += cnt[e];
    }
    CHECK(s == delta[r] && d32[r] == int32_t(uint32_t(uint64_t(delta[r]))));
    total += s;
  }
  CHECK(total == info.observed);
  // the same entries in row ranges: each range with an exact cap, then one short cap (refused, nothing written)
  std::vector<int32_t> rc(info.nnz + 1, -7);
  std::vector<uint32_t> rn(info.nnz + 1);
  for (int32_t r0 = 0; r0 < n; r0 += 7) {
    const int32_t r1 = r0 + 7 < n ? r0 + 7 : n;
    const int64_t m = rp[r1] - rp[r0];
    OK(cooc_copy_window_delta_range(ctx, r0, r1, m, rc.data(), rn.data(), nullptr));
    for (int64_t e = 0; e < m; e++) CHECK(rc[e] == cols[rp[r0] + e] && rn[e] == cnt[rp[r0] + e]);
    if (m > 0) {
      rc[m - 1] = -7;
      CHECK(cooc_copy_window_delta_range(ctx, r0, r1, m - 1, rc.data(), rn.data(), nullptr) == COOC_ERR_ARG);
      CHECK(rc[m - 1] == -7);
    }
  }
  CHECK(cooc_copy_window_delta_range(ctx, n, n + 1, 1 << 20, rc.data(), rn.data(), nullptr) != 0);
  CHECK(cooc_copy_window_delta_range(ctx, 1, 0, 1 << 20, rc.data(), rn.data(), nullptr) != 0);
  if (topk > 0 && info.n_topk > 0) {
    std::vector<int32_t> trows(info.n_topk), sizes(info.n_topk), vals(size_t(info.n_topk) * topk);
    std::vector<double> scores(size_t(info.n_topk) * topk);
    OK(cooc_copy_window_topk(ctx, trows.data(), sizes.data(), vals.data(), scores.data()));
    for (int32_t i = 0; i < info.n_topk; i++) {
      CHECK(sizes[i] >= 0 && sizes[i] <= topk);
      for (int32_t j = 0; j < sizes[i]; j++) CHECK(vals[size_t(i) * topk + j] >= 0 && vals[size_t(i) * topk + j] < M);
    }
  }
  g_windows++;
  g_entries += info.nnz;
}

void run(int32_t M, int32_t U, int64_t n_rec, uint64_t seed, int32_t topk, int32_t flags) {
  cooc_config cfg{};
  cfg.device = 0;
  cfg.n_items = M;
  cfg.topk = topk;
  cfg.flags = flags;
  cfg.window_size_ms = 1000;
  cooc_ctx *ctx = nullptr;
  if (cooc_create(&cfg, &ctx) != 0) {
    std::fprintf(stderr, "cooc_create failed\n");
    std::exit(1);
  }
  std::mt19937_64 rng(seed);
  std::vector<int32_t> users(n_rec), items(n_rec);
  std::vector<int64_t> ts(n_rec);
  int64_t t = 0;
  for (int64_t i = 0; i < n_rec; i++) {
    users[i] = int32_t(rng() % uint64_t(U));
    // Zipf-ish items: a small power of a uniform draw keeps the head hot
    const double x = double(rng() >> 11) * (1.0 / 9007199254740992.0);
    items[i] = int32_t(double(M) * x * x * x) % M;
    t += int64_t(rng() % 3);
    if (i % 5000 == 4999) t += 4000;  // a gap: empty windows in between
    ts[i] = t;
  }
  int64_t late_total = 0, fired_total = 0, observed = 0;
  const int64_t chunk = 1500;
  for (int64_t lo = 0; lo < n_rec; lo += chunk) {
    const int64_t n = lo + chunk < n_rec ? chunk : n_rec - lo;
    int64_t late = 0;
    OK(cooc_op_process_elements(ctx, n, users.data() + lo, items.data() + lo, ts.data() + lo, &late));
    late_total += late;
    // every other chunk also replays a few old records (late: dropped and counted)
    if ((lo / chunk) % 2 == 1 && lo >= chunk) {
      OK(cooc_op_process_elements(ctx, 16, users.data(), items.data(), ts.data(), &late));
      late_total += late;
    }
    if (lo == 0) {  // an item outside [0, n_items) in a record that is not late: refused
      const int32_t bad_item = M, u0 = 0;
      const int64_t ts0 = ts[n - 1] + 1;
      CHECK(cooc_op_process_elements(ctx, 1, &u0, &bad_item, &ts0, &late) == COOC_ERR_ARG);
    }
    for (;;) {
      int32_t fired = 0;
      cooc_window_info info{};
      OK(cooc_op_process_watermark(ctx, ts[lo + n - 1] - 1, &fired, &info));
      if (!fired) break;
      fired_total++;
      observed += info.observed;
      read_window(ctx, info, M, topk);
    }
  }
  for (;;) {
    int32_t fired = 0;
    cooc_window_info info{};
    OK(cooc_op_process_watermark(ctx, INT64_MAX, &fired, &info));
    if (!fired) break;
    fired_total++;
    observed += info.observed;
    read_window(ctx, info, M, topk);
  }
  int64_t counters[5];
  OK(cooc_op_counters(ctx, counters));
  CHECK(counters[0] == late_total && counters[1] == observed);
  std::vector<int64_t> gx(M);
  std::vector<int32_t> g32(M);
  OK(cooc_global_rowsums(ctx, gx.data(), g32.data()));
  int64_t gsum = 0;
  for (int32_t a = 0; a < M; a++) gsum += gx[a];
  CHECK(gsum == observed);
  int64_t ex = 0, resc = 0;
  OK(cooc_global_observed(ctx, &ex, &resc));
  CHECK(ex == observed);
  for (int32_t a = 0; a < M; a += M / 97 + 1) {
    int64_t nnz = -1;
    OK(cooc_global_row_nnz(ctx, a, &nnz));
    std::vector<int32_t> c(nnz + 1);
    std::vector<uint32_t> v(nnz + 1);
    std::vector<int16_t> v16(nnz + 1);
    OK(cooc_global_row(ctx, a, c.data(), v.data(), v16.data()));
    int64_t s = 0;
    for (int64_t e = 0; e < nnz; e++) s += v[e];
    CHECK(s == gx[a]);
  }
  // invalid arguments are refused with an error, not a crash
  int64_t nnz = 0;
  CHECK(cooc_global_row_nnz(ctx, M, &nnz) != 0);
  CHECK(cooc_global_row_nnz(ctx, -1, &nnz) != 0);
  std::printf("M %d: %lld windows fired, %lld late\n", M, (long long)fired_total, (long long)late_total);
  cooc_destroy(ctx);
}

}  // namespace

int main() {
  run(300, 400, 40000, 1, 10, 0);         // dense-tile windows (small universe)
  run(60000, 3000, 60000, 2, 10, 0);      // large-universe windows
  run(300, 50, 20000, 3, 0, 0);           // no rescoring; long histories
  CHECK(g_windows > 20);
  std::printf("stream_asan ok (%lld windows, %lld entries)\n", (long long)g_windows, (long long)g_entries);
  return 0;
}
