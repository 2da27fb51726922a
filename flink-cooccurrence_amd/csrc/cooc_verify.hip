// cooc_verify.hip — invariant checks and per-row fingerprints of a batch result (cooc_verify_batch).
//
// The reference checks its own state only in DEVELOPMENT_MODE (FlinkCooccurrences.java:34): the sum
// of a global row must equal the item's row sum (ItemRowRescorer...java:183-193).  These kernels run
// that check, and the ones the CSR contract adds, over a whole cooc_count_device result in HBM:
//   * sum over the row's counts == rowsum[a] (the closed form W_a - c_a the planner wrote),
//   * columns strictly ascending within a row (in the result's column order: ascending rank_of[col] after the
//     large-universe path's frequency relabel, else ascending id; not checked for a COOC_FLAG_ANY_ORDER
//     result) and inside [0, n_items), every stored
//     count > 0
//     (a key exists iff it was touched: every increment is +1, ItemRowAggregator.java:29),
//   * optionally C[a, b] == C[b, a] for every entry (the ordered pairs of a user are symmetric),
// and write a per-row fingerprint, sum over the row's keys of splitmix64(col << 32 ^ count) mod 2^64,
// that a test or the benchmark compares with an independent CPU restatement of the same rows
// (oracle/cooc_oracle.c, oc_row_checksums) without copying the matrix out.
#include "cooc_device.h"
#include "cooc_scan.h"
#include "cooc_radix.h"

#include <algorithm>

namespace cooc {

namespace {

__device__ inline uint64_t row_key_hash(int32_t col, uint64_t count) {
  uint64_t x = (uint64_t(uint32_t(col)) << 32) ^ count;
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ inline uint64_t wave_sum(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// tot: [0] sum of counts, [1] sum of row sums, [2] entries, [3] rows whose counts miss the row sum,
// [4] rows with a bad entry (order, range, zero count), [5] asymmetric entries.
// Padded CSR: one wave per row.
__global__ __launch_bounds__(256) void k_verify_csr(int32_t M, const int64_t *__restrict__ row_base,
                                                    const int32_t *__restrict__ row_nnz, const int32_t *__restrict__ col,
                                                    const uint32_t *__restrict__ cnt, const int64_t *__restrict__ rowsum,
                                                    const int32_t *__restrict__ rank_of, int32_t ordered,
                                                    uint64_t *__restrict__ cs_out, unsigned long long *__restrict__ tot) {
  const int lane = threadIdx.x & 63;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  uint64_t t_sum = 0, t_rs = 0, t_nnz = 0, t_badsum = 0, t_bad = 0;
  for (int64_t a = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; a < M; a += n_waves) {
    const int32_t n = row_nnz[a];
    const int64_t b = n > 0 ? row_base[a] : 0;
    uint64_t h = 0, s = 0, bad = 0;
    for (int32_t i = lane; i < n; i += 64) {
      const int32_t c = col[b + i];
      const uint32_t v = cnt[b + i];
      h += row_key_hash(c, v);
      s += v;
      bool ok = c >= 0 && c < M && v > 0u;
      if (ok && ordered && i + 1 < n) {
        const int32_t c1 = col[b + i + 1];
        ok = rank_of ? (c1 >= 0 && c1 < M && rank_of[c1] > rank_of[c]) : c1 > c;
      }
      bad += ok ? 0u : 1u;
    }
    h = wave_sum(h);
    s = wave_sum(s);
    bad = wave_sum(bad);
    if (lane == 0) {
      if (cs_out) cs_out[a] = h;
      const uint64_t rs = uint64_t(rowsum[a]);
      t_sum += s;
      t_rs += rs;
      t_nnz += uint64_t(n < 0 ? 0 : n);
      t_badsum += s != rs;
      t_bad += (bad != 0) || n < 0;
    }
  }
  if (lane == 0) {
    if (t_sum) atomicAdd(tot + 0, (unsigned long long)t_sum);
    if (t_rs) atomicAdd(tot + 1, (unsigned long long)t_rs);
    if (t_nnz) atomicAdd(tot + 2, (unsigned long long)t_nnz);
    if (t_badsum) atomicAdd(tot + 3, (unsigned long long)t_badsum);
    if (t_bad) atomicAdd(tot + 4, (unsigned long long)t_bad);
  }
}

// Dense [M x M] result: one wave per row; row_nnz[a] is checked against the row's non-zero cells.
__global__ __launch_bounds__(256) void k_verify_dense(int32_t M, const uint32_t *__restrict__ dense,
                                                      const int32_t *__restrict__ row_nnz,
                                                      const int64_t *__restrict__ rowsum, uint64_t *__restrict__ cs_out,
                                                      unsigned long long *__restrict__ tot) {
  const int lane = threadIdx.x & 63;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  uint64_t t_sum = 0, t_rs = 0, t_nnz = 0, t_badsum = 0, t_bad = 0;
  for (int64_t a = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; a < M; a += n_waves) {
    const uint32_t *row = dense + a * int64_t(M);
    uint64_t h = 0, s = 0, nz = 0;
    for (int32_t c = lane; c < M; c += 64) {
      const uint32_t v = row[c];
      if (v) {
        h += row_key_hash(c, v);
        s += v;
        nz++;
      }
    }
    h = wave_sum(h);
    s = wave_sum(s);
    nz = wave_sum(nz);
    if (lane == 0) {
      if (cs_out) cs_out[a] = h;
      const uint64_t rs = uint64_t(rowsum[a]);
      t_sum += s;
      t_rs += rs;
      t_nnz += nz;
      t_badsum += s != rs;
      t_bad += nz != uint64_t(row_nnz[a]);
    }
  }
  if (lane == 0) {
    if (t_sum) atomicAdd(tot + 0, (unsigned long long)t_sum);
    if (t_rs) atomicAdd(tot + 1, (unsigned long long)t_rs);
    if (t_nnz) atomicAdd(tot + 2, (unsigned long long)t_nnz);
    if (t_badsum) atomicAdd(tot + 3, (unsigned long long)t_badsum);
    if (t_bad) atomicAdd(tot + 4, (unsigned long long)t_bad);
  }
}

// C[a, b] == C[b, a] for every entry of the padded CSR: one wave per row a, every lane looks its
// entry's column b up in row b (binary search; rows are sorted, k_verify_csr checks that).
__global__ __launch_bounds__(256) void k_verify_symmetry(int32_t M, const int64_t *__restrict__ row_base,
                                                         const int32_t *__restrict__ row_nnz,
                                                         const int32_t *__restrict__ col,
                                                         const uint32_t *__restrict__ cnt,
                                                         const int32_t *__restrict__ rank_of,
                                                         unsigned long long *__restrict__ tot) {
  const int lane = threadIdx.x & 63;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  uint64_t bad = 0;
  for (int64_t a = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; a < M; a += n_waves) {
    const int32_t n = row_nnz[a];
    const int64_t base = n > 0 ? row_base[a] : 0;
    for (int32_t i = lane; i < n; i += 64) {
      const int32_t b = col[base + i];
      const uint32_t v = cnt[base + i];
      if (b < 0 || b >= M) {
        bad++;
        continue;
      }
      const int32_t nb = row_nnz[b];
      const int64_t bb = nb > 0 ? row_base[b] : 0;
      // (rows are sorted in the result's column order, k_verify_csr checks that)
      const int32_t ka = rank_of ? rank_of[a] : int32_t(a);
      int32_t lo = 0, hi = nb;
      while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        const int32_t cm = col[bb + mid];
        if ((rank_of ? rank_of[cm] : cm) < ka) lo = mid + 1; else hi = mid;
      }
      bad += !(lo < nb && col[bb + lo] == int32_t(a) && cnt[bb + lo] == v);
    }
  }
  bad = wave_sum(bad);
  if (lane == 0 && bad) atomicAdd(tot + 5, (unsigned long long)bad);
}

}  // namespace

Status launch_verify(hipStream_t s, int32_t M, const CountResult &r, bool symmetry, uint64_t *d_cs,
                     unsigned long long *d_tot) {
  COOC_HIP_TRY(hipMemsetAsync(d_tot, 0, sizeof(unsigned long long) * 8, s));
  if (M <= 0) return Status::Ok();
  const unsigned grid = unsigned(std::min<int64_t>((int64_t(M) * 64 + 255) / 256, 8192));
  if (r.dense) {
    k_verify_dense<<<grid, 256, 0, s>>>(M, r.dense, r.row_nnz, r.rowsum, d_cs, d_tot);
  } else {
    k_verify_csr<<<grid, 256, 0, s>>>(M, r.row_base, r.row_nnz, r.col, r.cnt, r.rowsum, r.rank_of, r.unordered ? 0 : 1,
                                      d_cs, d_tot);
    if (symmetry && !r.unordered) k_verify_symmetry<<<grid, 256, 0, s>>>(M, r.row_base, r.row_nnz, r.col, r.cnt, r.rank_of, d_tot);
  }
  COOC_HIP_TRY(hipGetLastError());
  return Status::Ok();
}

// The planner's device prefix sum (cooc_scan.h) on a caller's array, every variant the library uses: inclusive /
// exclusive, vectorised or LDS-staged tiles, int64 / int32 input and output (cooc_selftest_scan).
Status selftest_scan(const void *d_in, void *d_out, int64_t n, int32_t flags, hipStream_t s, int64_t *h_err) {
  *h_err = 0;
  if (n <= 0) return Status::Ok();
  unsigned long long *ws = nullptr;
  COOC_HIP_TRY(hipMalloc(&ws, scan_ws_bytes(n)));
  const int blocked = (flags & 2) ? 0 : 1;
  const bool incl = flags & 1, out32 = flags & 4, in32 = flags & 8;
  int64_t *err = reinterpret_cast<int64_t *>(ws + scan_state_words(n));
  Status st = Status::Ok();
  if (hipMemsetAsync(err, 0, sizeof(int64_t), s) != hipSuccess) st = Status{3, "hipMemsetAsync"};
  auto run = [&](auto in) {
    if (!st.ok()) return;
    if (incl && out32) st = launch_scan<true>(in, static_cast<int32_t *>(d_out), n, ws, err, s, blocked);
    else if (incl) st = launch_scan<true>(in, static_cast<int64_t *>(d_out), n, ws, err, s, blocked);
    else if (out32) st = launch_scan<false>(in, static_cast<int32_t *>(d_out), n, ws, err, s, blocked);
    else st = launch_scan<false>(in, static_cast<int64_t *>(d_out), n, ws, err, s, blocked);
  };
  if (in32) run(ScanI32{static_cast<const int32_t *>(d_in)});
  else run(ScanI64{static_cast<const int64_t *>(d_in)});
  if (st.ok() && hipMemcpyAsync(h_err, err, sizeof(int64_t), hipMemcpyDeviceToHost, s) != hipSuccess)
    st = Status{3, "hipMemcpyAsync"};
  if (st.ok() && hipStreamSynchronize(s) != hipSuccess) st = Status{3, "hipStreamSynchronize"};
  (void)hipFree(ws);
  return st;
}

// The planner's radix sort (cooc_radix.h) on a caller's arrays: 32- or 64-bit keys, 32-bit values, any bit range,
// ascending or descending (cooc_selftest_radix); and its flag compaction (cooc_selftest_select).
Status selftest_radix(const void *kin, const void *vin, void *kout, void *vout, int64_t n, int32_t key_bytes,
                      int32_t bit0, int32_t bit1, int32_t desc, hipStream_t s) {
  if (n <= 0) return Status::Ok();
  void *tmp = nullptr;
  const size_t bytes = key_bytes == 8 ? radix_sort_tmp_bytes<uint64_t, uint32_t>(n) : radix_sort_tmp_bytes<uint32_t, uint32_t>(n);
  COOC_HIP_TRY(hipMalloc(&tmp, bytes));
  Status st = key_bytes == 8
                  ? radix_sort_pairs(static_cast<const uint64_t *>(kin), static_cast<const uint32_t *>(vin),
                                     static_cast<uint64_t *>(kout), static_cast<uint32_t *>(vout), n, bit0, bit1,
                                     desc != 0, tmp, s)
                  : radix_sort_pairs(static_cast<const uint32_t *>(kin), static_cast<const uint32_t *>(vin),
                                     static_cast<uint32_t *>(kout), static_cast<uint32_t *>(vout), n, bit0, bit1,
                                     desc != 0, tmp, s);
  if (st.ok() && hipStreamSynchronize(s) != hipSuccess) st = Status{3, "hipStreamSynchronize"};
  (void)hipFree(tmp);
  return st;
}
Status selftest_select(const uint8_t *flag, int64_t n, int32_t *out, int32_t *n_sel, hipStream_t s) {
  void *tmp = nullptr;
  COOC_HIP_TRY(hipMalloc(&tmp, select_tmp_bytes(std::max<int64_t>(n, 1))));
  Status st = select_flagged(flag, n, out, n_sel, tmp, s);
  if (st.ok() && hipStreamSynchronize(s) != hipSuccess) st = Status{3, "hipStreamSynchronize"};
  (void)hipFree(tmp);
  return st;
}

}  // namespace cooc
