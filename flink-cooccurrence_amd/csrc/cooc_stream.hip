// cooc_stream.hip — kernels of the resident streaming state.
//
//   k_relocate / k_append   per-user history arena (NonSampled...java:129-161: userHistory.add)
//   k_merge_global          global rows += window delta rows (ItemRowRescorer...java:171-177),
//                           global row sums += row-sum deltas and the rescorer's observed total
//                           += the int view of every delta (:144-156)
//   k_rescore               LLR of every entry of every touched row + top-k heap
//                           (ItemRowRescorer...java:195-241, LogLikelihood.java:41-61,
//                           IntDoublePriorityQueue.java:132-205), rows iterated in column order
//
// Compiled with -ffp-contract=off: the LLR must keep Java's unfused operation order.
#include <hipcub/hipcub.hpp>

#include "cooc_stream_kernels.h"
#include "cooc_scan.h"

namespace cooc {
namespace {

inline unsigned blocks_for(int64_t n, int t) { return unsigned((n + t - 1) / t); }

__global__ void k_relocate(int64_t n, const int64_t *__restrict__ reloc, int32_t *__restrict__ arena) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t r = wave; r < n; r += n_waves) {
    const int64_t src = reloc[3 * r], dst = reloc[3 * r + 1], len = reloc[3 * r + 2];
    for (int64_t i = lane; i < len; i += 64) arena[dst + i] = arena[src + i];
  }
}

__global__ void k_append(int64_t n, const int64_t *__restrict__ new_ptr, const int64_t *__restrict__ new_dst,
                         const int32_t *__restrict__ new_items, int32_t *__restrict__ arena) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t j = wave; j < n; j += n_waves) {
    const int64_t s = new_ptr[j], e = new_ptr[j + 1], d = new_dst[j];
    for (int64_t i = s + lane; i < e; i += 64) arena[d + (i - s)] = new_items[i];
  }
}

// Contiguous copies of arena slabs: list j (len[j] ids at off[j]) to out[dst[j] ..).  One wave per list.
__global__ void k_gather_lists(int64_t n, const int64_t *__restrict__ off, const int32_t *__restrict__ len,
                               const int64_t *__restrict__ dst, const int32_t *__restrict__ arena,
                               int32_t *__restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t j = wave; j < n; j += n_waves) {
    const int64_t s = off[j], d = dst[j];
    for (int64_t i = lane; i < len[j]; i += 64) out[d + i] = arena[s + i];
  }
}

// kMax cap (UserInteractionCounter...java:168): capped length min(n_u, cut) of every user at
// lens[u + 1]; an inclusive scan of lens[1..U] gives the capped offsets.
__global__ void k_cut_lens(int64_t U, const int64_t *__restrict__ up, int32_t cut, int64_t *__restrict__ lens) {
  const int64_t u = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (u < U) lens[u + 1] = min(up[u + 1] - up[u], int64_t(cut));
}

// One wave per user copies its first (capped) items; the source rows are read coalesced.
__global__ void k_cut_copy(int64_t U, const int64_t *__restrict__ up, const int32_t *__restrict__ items,
                           const int64_t *__restrict__ cut_ptr, int32_t *__restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t u = wave; u < U; u += n_waves) {
    const int64_t s = up[u], d = cut_ptr[u], n = cut_ptr[u + 1] - d;
    for (int64_t i = lane; i < n; i += 64) out[d + i] = items[s + i];
  }
}

// One wave per row with a non-empty delta; the int views of the row-sum deltas are summed per
// workgroup (one global atomic per workgroup, not per row).
__global__ __launch_bounds__(256) void k_merge_global(int32_t M, const int64_t *__restrict__ row_base,
                                                      const int32_t *__restrict__ row_nnz,
                                                      const int32_t *__restrict__ col, const uint32_t *__restrict__ cnt,
                                                      const int64_t *__restrict__ rowsum_delta,
                                                      uint32_t *__restrict__ G, int64_t *__restrict__ grs,
                                                      int64_t *__restrict__ scal) {
  __shared__ int64_t s_d32[4];
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  int64_t d32 = 0;
  for (int64_t a = wave; a < M; a += n_waves) {
    const int32_t n = row_nnz[a];
    if (n == 0) continue;
    const int64_t b = row_base[a];
    if (G) {  // dense global rows (sparse ones are merged by k_gs_flags / k_gs_move_all / k_gs_insert)
      uint32_t *g = G + a * int64_t(M);
      for (int32_t i = lane; i < n; i += 64) g[col[b + i]] += cnt[b + i];  // unique (a, col) per window
    }
    if (lane == 0 && rowsum_delta) {
      const int64_t d = rowsum_delta[a];
      grs[a] += d;
      d32 += int64_t(int32_t(uint32_t(uint64_t(d))));  // RowSumAggregator's int value, ItemRowRescorer...java:154
    }
  }
  if (lane == 0) s_d32[threadIdx.x >> 6] = d32;
  __syncthreads();
  if (threadIdx.x == 0 && scal) {
    const int64_t t = s_d32[0] + s_d32[1] + s_d32[2] + s_d32[3];
    if (t) atomicAdd(reinterpret_cast<unsigned long long *>(scal + 1), (unsigned long long)t);
  }
}

__global__ void k_finish_scalars(int64_t *__restrict__ scal, int64_t observed_window) {
  scal[2] += scal[1];
  scal[3] += observed_window;
}

// ---- multi-GPU windows (p > 1 subtasks, the keyBy(item) of FlinkCooccurrences.java:152): after the owner
// merged its rows' partial deltas (Sharder::merge: rows a = part + r W), the M-row view of them, their merge
// into the resident rows, every item's all-reduced row-sum delta, and the packed copy-out.
__global__ void k_own_scatter(int32_t R, int32_t W, int32_t part, const int64_t *__restrict__ mbase,
                              const int32_t *__restrict__ mnnz, int64_t *__restrict__ base, int32_t *__restrict__ nnz) {
  const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const int64_t a = int64_t(part) + int64_t(r) * W;
  base[a] = mbase[r];
  nnz[a] = mnnz[r];
}

// every item's window row sum (all-reduced: the broadcast row-sum stream, :163) into the global row sums; scal[1]
// = the sum of their int views over ALL items (the rescorer's observed, :154), scal[4] = over the OWNED rows with
// a delta only (this subtask's RowSumProcessWindowRowSum accumulator, RowSumAggregator.java:50,67)
__global__ __launch_bounds__(256) void k_add_rowsums(int32_t M, const int64_t *__restrict__ rs, const int32_t *__restrict__ nnz,
                                                     int64_t *__restrict__ grs, int64_t *__restrict__ scal) {
  __shared__ int64_t s_all[4], s_own[4];
  int64_t all = 0, own = 0;
  for (int64_t a = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; a < M; a += int64_t(gridDim.x) * blockDim.x) {
    const int64_t d = rs[a];
    if (d == 0) continue;
    grs[a] += d;
    const int64_t d32 = int64_t(int32_t(uint32_t(uint64_t(d))));
    all += d32;
    if (nnz[a] > 0) own += d32;
  }
  for (int o = 32; o > 0; o >>= 1) {
    all += __shfl_xor(all, o, 64);
    own += __shfl_xor(own, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    s_all[threadIdx.x >> 6] = all;
    s_own[threadIdx.x >> 6] = own;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t t = s_all[0] + s_all[1] + s_all[2] + s_all[3], u = s_own[0] + s_own[1] + s_own[2] + s_own[3];
    if (t) atomicAdd(reinterpret_cast<unsigned long long *>(scal + 1), (unsigned long long)t);
    if (u) atomicAdd(reinterpret_cast<unsigned long long *>(scal + 4), (unsigned long long)u);
  }
}

// one wave per row: the row's entries copied to its packed offset rp[a]
__global__ __launch_bounds__(256) void k_pack_rows(int32_t M, const int64_t *__restrict__ base, const int32_t *__restrict__ nnz,
                                                   const int64_t *__restrict__ rp, const int32_t *__restrict__ col,
                                                   const uint32_t *__restrict__ cnt, int32_t *__restrict__ out_col,
                                                   uint32_t *__restrict__ out_cnt) {
  const int lane = threadIdx.x & 63;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t a = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; a < M; a += n_waves) {
    const int32_t n = nnz[a];
    const int64_t b = base[a], o = rp[a];
    for (int32_t i = lane; i < n; i += 64) {
      out_col[o + i] = col[b + i];
      out_cnt[o + i] = cnt[b + i];
    }
  }
}

struct IsTouched {
  const int32_t *row_nnz;
  __host__ __device__ bool operator()(int32_t a) const { return row_nnz[a] > 0; }
};

// ---- LogLikelihood.java:41-61 (Java operation order, no contraction) -------------------------
// Math.log (LogLikelihood.java:60) as Java's StrictMath.log pins it: fdlibm 5.3's __ieee754_log (Java's Math.log
// may differ from it by at most one ulp; StrictMath.log is exactly this function).  x = 2^k (1 + f) with
// sqrt(2)/2 <= 1 + f < sqrt(2), s = f / (2 + f), log(1 + f) = f - s (f - R(s^2)) with fdlibm's degree-14 Remez
// polynomial (Lg1..Lg7), k ln2 as ln2_hi + ln2_lo, in fdlibm's operation order and without contraction, so the
// device's scores equal the oracle's restatement (oracle/cooc_oracle.c, strict_log) bit for bit.
__device__ inline double java_log(double x) {
#pragma clang fp contract(off)
  constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                   two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
                   Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                   Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
  uint64_t u = uint64_t(__double_as_longlong(x));
  int32_t hx = int32_t(u >> 32);
  int32_t k = 0;
  if (hx < 0x00100000) {  // x < 2^-1022: zero, negative or subnormal
    if (((hx & 0x7fffffff) | int32_t(uint32_t(u))) == 0) return -__builtin_inf();
    if (hx < 0) return __builtin_nan("");
    k -= 54;
    u = uint64_t(__double_as_longlong(x * two54));
    hx = int32_t(u >> 32);
  }
  if (hx >= 0x7ff00000) {
    const double y = __longlong_as_double(int64_t(u));
    return y + y;
  }
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  const int32_t i0 = (hx + 0x95f64) & 0x100000;
  u = (uint64_t(uint32_t(hx | (i0 ^ 0x3ff00000))) << 32) | (u & 0xffffffffull);  // x or x/2 into [sqrt2/2, sqrt2)
  k += i0 >> 20;
  const double f = __longlong_as_double(int64_t(u)) - 1.0;
  const double dk = double(k);
  if ((0x000fffff & (2 + hx)) < 3) {  // |f| < 2^-20
    if (f == 0.0) return k == 0 ? 0.0 : dk * ln2_hi + dk * ln2_lo;
    const double R = f * f * (0.5 - 0.33333333333333333 * f);
    return k == 0 ? f - R : dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  const double s = f / (2.0 + f);
  const double z = s * s;
  const double w = z * z;
  const int32_t i = (hx - 0x6147a) | (0x6b851 - hx);
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  const double R = t2 + t1;
  if (i > 0) {
    const double hfsq = 0.5 * f * f;
    return k == 0 ? f - (hfsq - s * (hfsq + R)) : dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  return k == 0 ? f - s * (f - R) : dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

__device__ inline double xlogx(int64_t x) {
#pragma clang fp contract(off)
  return x == 0 ? 0.0 : double(x) * java_log(double(x));
}

__device__ inline double llr(int64_t k11, int64_t k12, int64_t k21, int64_t k22) {
#pragma clang fp contract(off)
  const int64_t k11k12 = k11 + k12;
  const int64_t k21k22 = k21 + k22;
  const double all = xlogx(k11k12 + k21k22);
  const double row = all - xlogx(k11k12) - xlogx(k21k22);
  const double column = all - xlogx(k11 + k21) - xlogx(k12 + k22);
  const double matrix = all - xlogx(k11) - xlogx(k12) - xlogx(k21) - xlogx(k22);
  if (row + column < matrix) return 0.0;
  return 2.0 * (row + column - matrix);
}

// The same function over precomputed x log x terms, in the same operation order (bit-identical when
// every term is: a term looked up from a table was computed by the same xlogx of the same integer).
__device__ inline double llr_terms(double all, double x_k11k12, double x_k21k22, double x_k11k21, double x_k12k22,
                                   double x_k11, double x_k12, double x_k21, double x_k22) {
#pragma clang fp contract(off)
  const double row = all - x_k11k12 - x_k21k22;
  const double column = all - x_k11k21 - x_k12k22;
  const double matrix = all - x_k11 - x_k12 - x_k21 - x_k22;
  if (row + column < matrix) return 0.0;
  return 2.0 * (row + column - matrix);
}

// Per column b of the rescored rows (the int32 view of its row sum unless exact): rs = rowSum(b) and the
// terms of an entry with k11 == 1 that depend on b only (ItemRowRescorer...java:230-240): k11 + k21 =
// rs, k21 = rs - 1, k12 + k22 = observed + 2 - rs.  32 B per column, one line per gathered entry.
constexpr int kRsR = 8;  // 64-entry steps scored before the heap is fed (per wave)
constexpr int64_t kRsChunk = kRsR * 64;
struct alignas(32) ColTerms {
  int64_t rs;
  double x_rs;   // xlogx(rs)
  double x_rs1;  // xlogx(rs - 1)
  double x_or2;  // xlogx(observed + 2 - rs)
};

__global__ void k_col_terms(int32_t M, const int64_t *__restrict__ grs, const int64_t *__restrict__ obs, int32_t exact,
                            ColTerms *__restrict__ out) {
  const int32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= M) return;
  const int64_t observed = exact ? obs[1] : obs[0];
  const int64_t rs = exact ? grs[b] : int64_t(int32_t(uint32_t(uint64_t(grs[b]))));
  out[b] = ColTerms{rs, xlogx(rs), xlogx(rs - 1), xlogx(observed + 2 - rs)};
}

// xlogx(k11) and xlogx(observed + 2 k11) for every int16 k11 (index k11 + 32768; the second table at
// + 65536): the two terms of the full LLR that depend on the count alone.
__global__ void k_k11_terms(const int64_t *__restrict__ obs, int32_t exact, double *__restrict__ out) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 65536) return;
  const int64_t observed = exact ? obs[1] : obs[0];
  const int64_t k11 = int64_t(i) - 32768;
  out[i] = xlogx(k11);
  out[i + 65536] = xlogx(observed + 2 * k11);
}

// ---- IntDoublePriorityQueue.java:132-205, every lane of the wave runs it on the same LDS heap ----
__device__ inline void heap_add(int32_t *hv, double *hs, int32_t &size, int32_t value, double score) {
  size++;
  int32_t i = size;
  int32_t j = i >> 1;
  while (j > 0 && score < hs[j]) {
    hv[i] = hv[j];
    hs[i] = hs[j];
    i = j;
    j = j >> 1;
  }
  hv[i] = value;
  hs[i] = score;
}

__device__ inline void heap_update(int32_t *hv, double *hs, int32_t size, int32_t value, double score) {
  int32_t i = 1, j = 2, k = 3;
  if (k <= size && hs[k] < hs[j]) j = k;
  while (j <= size && hs[j] < score) {
    hv[i] = hv[j];
    hs[i] = hs[j];
    i = j;
    j = i << 1;
    k = j + 1;
    if (k <= size && hs[k] < hs[j]) j = k;
  }
  hv[i] = value;
  hs[i] = score;
}

// Row sources for the rescoring kernel: a dense global row (streaming state) or a padded CSR row
// (a batch result).  Both are iterated in ascending column order (the tie contract).
struct DenseRows {
  const uint32_t *G;
  int32_t M;
  __device__ int64_t size(int32_t) const { return M; }
  __device__ int64_t base(int32_t a) const { return int64_t(a) * M; }
  __device__ void get_at(int64_t b, int64_t i, int32_t &c, uint32_t &v) const {
    c = int32_t(i);
    v = G[b + i];
  }
};

struct CsrRows {
  const int64_t *row_base;
  const int32_t *row_nnz;
  const int32_t *col;
  const uint32_t *cnt;
  __device__ int64_t size(int32_t a) const { return row_nnz[a]; }
  __device__ int64_t base(int32_t a) const { return row_base[a]; }
  __device__ void get_at(int64_t b, int64_t i, int32_t &c, uint32_t &v) const {
    c = col[b + i];
    v = cnt[b + i];
  }
};

// Per-row constants of the rescorer's LLR (ItemRowRescorer...java:199-205): k11k12 = k11 + k12 = rs_a;
// with k11 == 1 also k11k12 + k21k22 = observed + 2, k21k22 = observed + 2 - rs_a, k12 = rs_a - 1.
struct RowTerms {
  int64_t observed, rs_a;
  double x_a, x_all1, x_r1, x_a1;
  __device__ RowTerms(int64_t obs, int64_t rs) : observed(obs), rs_a(rs) {
    x_a = xlogx(rs);
    x_all1 = xlogx(obs + 2);
    x_r1 = xlogx(obs + 2 - rs);
    x_a1 = xlogx(rs - 1);
  }
};

// Scores the kRsR * 64 entries [i0, i0 + kRsR * 64) of row a into the wave's LDS ring: rscore[k] = the
// entry's LLR, rcol[k] = its column (-1: no entry or a zero count).  Scoring is split by count so that
// the wave's lanes do not diverge over the expensive case: an entry with k11 == 1 (most of a sparse
// row) needs one log (every other term comes from the per-column table and the row's constants); the
// others (hot pairs, wrapped or zero int16 views) are queued in LDS and scored 64 at a time with the
// full formula (5 logs; the two terms that depend on k11 alone come from k_k11_terms' tables).  Both
// are LogLikelihood.java:41-57 in Java's operation order, bit for bit.
// The full formula's xlogx(k12) = xlogx(rs_a - k11) and xlogx(k21 + k22) = xlogx(observed + 2 k11 - rs_a) depend
// on the row and k11 only: the row's LDS tables over k11 < kRsK (tr12, tr2122) hold them, and xlogx(k21) of a
// column with |rs_b - k11| < 32768 is a k11t entry -- the same function of the same integer, so the same bits.
constexpr int kRsK = 64;
template <class Rows>
__device__ inline void rs_score_chunk(const Rows &src, int64_t rb, int64_t i0, int64_t n, const RowTerms &R,
                                      int32_t exact, const ColTerms *__restrict__ cterm,
                                      const double *__restrict__ k11t, const double *tr12, const double *tr2122,
                                      double *rscore, int32_t *rcol, int32_t *rq) {
  const int lane = threadIdx.x & 63;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t npend = 0;
  int32_t cj[kRsR];
  uint32_t vj[kRsR];
#pragma unroll
  for (int j = 0; j < kRsR; j++) {  // all kRsR steps' loads in flight at once (the row base hoisted by the caller)
    cj[j] = 0;
    vj[j] = 0u;
    if (i0 + j * 64 + lane < n) src.get_at(rb, i0 + j * 64 + lane, cj[j], vj[j]);
  }
  // the per-column terms of kRsG steps gathered before any of them is scored (their latency overlaps)
  constexpr int kRsG = 4;
#pragma unroll
  for (int j0 = 0; j0 < kRsR; j0 += kRsG) {
    ColTerms tg[kRsG];
#pragma unroll
    for (int g = 0; g < kRsG; g++) {
      const uint32_t v = vj[j0 + g];
      const int64_t k11 = exact ? int64_t(v) : int64_t(int16_t(uint16_t(v)));
      if (v != 0u && k11 == 1) tg[g] = cterm[cj[j0 + g]];
    }
#pragma unroll
    for (int g = 0; g < kRsG; g++) {
      const int j = j0 + g;
      const int32_t c = cj[j];
      const uint32_t v = vj[j];
      const int64_t k11 = exact ? int64_t(v) : int64_t(int16_t(uint16_t(v)));
      const bool fast = v != 0u && k11 == 1;
      double score = 0.0;
      if (fast) {  // ItemRowRescorer...java:203-205,230-240 (xlogx(1) = 0)
        const ColTerms &t = tg[g];
        const int64_t k22 = R.observed + k11 - (R.rs_a - k11) - (t.rs - k11);
        score = llr_terms(R.x_all1, R.x_a, R.x_r1, t.x_rs, t.x_or2, 0.0, R.x_a1, t.x_rs1, xlogx(k22));
      }
      const bool slow = v != 0u && !fast;
      const uint64_t sm = __ballot(slow);
      if (slow) rq[npend + uint32_t(__popcll(sm & lt))] = j * 64 + lane;
      npend += uint32_t(__popcll(sm));
      rscore[j * 64 + lane] = slow ? __longlong_as_double(k11) : score;  // slow: k11 parked until scored
      rcol[j * 64 + lane] = v != 0u ? c : -1;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  for (uint32_t p = lane; p < npend; p += 64) {  // LogLikelihood.java:41-57, k11k12 and k11 + k21 from tables
    const int32_t idx = rq[p];
    const int32_t c = rcol[idx];
    const int64_t k11 = __double_as_longlong(rscore[idx]);
    const ColTerms h = cterm[c];
    const int64_t k12 = R.rs_a - k11;
    const int64_t k21 = h.rs - k11;
    const int64_t k22 = R.observed + k11 - k12 - k21;
    // xlogx(k11) and xlogx(k11 + k12 + k21 + k22) = xlogx(observed + 2 k11) depend on k11 only: tables
    // over the int16 range (the same function, so the same bits)
    const bool in = k11 >= -32768 && k11 < 32768, inK = k11 >= 0 && k11 < kRsK;
    const double x_all = in ? k11t[k11 + 32768 + 65536] : xlogx(k11 + k12 + (k21 + k22));
    const double x_11 = in ? k11t[k11 + 32768] : xlogx(k11);
    const double x_12 = inK ? tr12[k11] : xlogx(k12);
    const double x_2122 = inK ? tr2122[k11] : xlogx(k21 + k22);
    const double x_21 = (k21 >= -32768 && k21 < 32768) ? k11t[k21 + 32768] : xlogx(k21);
    rscore[idx] = llr_terms(x_all, R.x_a, x_2122, h.x_rs, xlogx(k12 + k22), x_11, x_12, x_21, xlogx(k22));
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ inline int64_t rs_row_sum(const int64_t *__restrict__ grs, int32_t a, int32_t exact) {
  return exact ? grs[a] : int64_t(int32_t(uint32_t(uint64_t(grs[a]))));
}

// One wave per rescored row, taken from a counter (rows with long lists, the Zipf head, go first and
// no wave is left with a static share of them), rows iterated in ascending column order (the tie
// contract).  The wave scores kRsR steps of 64 entries (rs_score_chunk), then feeds the lanes that can
// enter the heap to it step by step in lane order, which is exactly the sequential loop of
// ItemRowRescorer...java:199-223.  rows == nullptr: rescored row t is item t.  obs[0] = the
// rescorer's observed (sum of int deltas), obs[1] = the exact pair count.
template <class Rows>
__global__ void k_rescore(const int32_t *__restrict__ rows, const int64_t *__restrict__ n_rows_p, Rows src,
                          const int64_t *__restrict__ grs, const ColTerms *__restrict__ cterm,
                          const double *__restrict__ k11t,
                          const int64_t *__restrict__ obs, int32_t exact, unsigned long long *__restrict__ row_ctr,
                          int32_t topk, int32_t *__restrict__ out_size, int32_t *__restrict__ out_val,
                          double *__restrict__ out_score, int32_t no_nan_exit, int32_t rbatch) {
  extern __shared__ double smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, waves = blockDim.x >> 6;
  double *hs = smem + int64_t(wave) * (topk + 1);
  int32_t *hv = reinterpret_cast<int32_t *>(smem + int64_t(waves) * (topk + 1)) + int64_t(wave) * (topk + 1);
  double *ring = smem + int64_t(waves) * (topk + 1) + (int64_t(waves) * (topk + 1) + 1) / 2;
  double *rscore = ring + int64_t(wave) * kRsChunk * 2;
  int32_t *rcol = reinterpret_cast<int32_t *>(rscore + kRsChunk);
  int32_t *rq = rcol + kRsChunk;
  double *tr12 = ring + int64_t(waves) * kRsChunk * 2 + int64_t(wave) * 2 * kRsK;
  double *tr2122 = tr12 + kRsK;
  const int64_t n_rows = n_rows_p[0];
  const int64_t observed = exact ? obs[1] : obs[0];
  // rows taken rbatch at a time from the counter (one atomic on one address per row costs more than a
  // short row's scoring once NaN roots end rows early)
  int64_t t_next = 0, t_end = 0;
  for (;;) {
    if (t_next == t_end) {
      t_next = __shfl(lane == 0 ? int64_t(atomicAdd(row_ctr, (unsigned long long)rbatch)) : 0ll, 0, 64);
      t_end = t_next + rbatch;
    }
    const int64_t t = t_next++;
    if (t >= n_rows) break;
    const int32_t a = rows ? rows[t] : int32_t(t);
    const RowTerms R(observed, rs_row_sum(grs, a, exact));
    const int64_t n = src.size(a);
    int32_t size = 0;
    double least = 0.0;
    const int64_t rb = n > 0 ? src.base(a) : 0;
    if (lane < kRsK) {  // (the previous row's reads of them are behind the wave barrier at its last chunk)
      tr12[lane] = xlogx(R.rs_a - lane);
      tr2122[lane] = xlogx(observed + 2 * int64_t(lane) - R.rs_a);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // the first chunk only as many 64-entry steps as fill the heap: a NaN root can end the row there
    const int64_t first = no_nan_exit ? kRsChunk : std::min<int64_t>(kRsChunk, (int64_t(topk) + 63) & ~int64_t(63));
    for (int64_t i0 = 0, span = first; i0 < n; i0 += span, span = kRsChunk) {
      const int64_t lim = std::min<int64_t>(n, i0 + span);
      rs_score_chunk(src, rb, i0, lim, R, exact, cterm, k11t, tr12, tr2122, rscore, rcol, rq);
      for (int j = 0; j < kRsR && i0 + j * 64 < lim; j++) {
        const int32_t c = rcol[j * 64 + lane];
        const double score = rscore[j * 64 + lane];
        uint64_t m = __ballot(c >= 0 && (size < topk || score > least));
        while (m) {
          const int l = __ffsll(static_cast<unsigned long long>(m)) - 1;
          m &= m - 1;
          const double sc = __shfl(score, l, 64);
          const int32_t cl = __shfl(c, l, 64);
          if (size < topk) {
            heap_add(hv, hs, size, cl, sc);
          } else if (sc > hs[1]) {
            heap_update(hv, hs, size, cl, sc);
          }
          least = hs[1];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // a full heap whose root (the least score) is NaN takes nothing more: the offer is score > least
      // (heap_update's test, IntDoublePriorityQueue.java:132-205), false against NaN, and nothing else
      // moves the root -- the rest of the row cannot change the heap, so it is not read (the wrapped int
      // views of a large window make nearly every root NaN)
      if (!no_nan_exit && size == topk && __builtin_isnan(least)) break;
    }
    out_size[t] = size;
    for (int32_t i = lane; i < size; i += 64) {
      out_val[t * topk + i] = hv[i + 1];
      out_score[t * topk + i] = hs[i + 1];
    }
  }
}

// The same rescoring, software-pipelined one 64-entry step at a time (the default; COOC_RS_V2=0 runs k_rescore):
// a row's step i is scored while the column terms of step i + 1 are gathered and the entries of step i + 2
// loaded, every lane scoring its own entry -- one log for k11 == 1, the full formula otherwise (the lanes of a
// step diverge over the two), both LogLikelihood.java:41-57 in Java's operation order with the same tables and
// the same fdlibm log as k_rescore, so the same bits -- and the step's entries that can enter the heap are fed to
// it in lane order (the sequential loop of ItemRowRescorer...java:199-223).  Without k_rescore's score ring and
// slow-entry queue a wave needs about half the registers: twice the waves per SIMD, each with a step of column
// terms in flight, where k_rescore's waves stalled on their gathers between scoring rounds.
template <class Rows>
__global__ __launch_bounds__(256) void k_rescore2(const int32_t *__restrict__ rows, const int64_t *__restrict__ n_rows_p,
                                                  Rows src, const int64_t *__restrict__ grs,
                                                  const ColTerms *__restrict__ cterm, const double *__restrict__ k11t,
                                                  const int64_t *__restrict__ obs, int32_t exact,
                                                  unsigned long long *__restrict__ row_ctr, int32_t topk,
                                                  int32_t *__restrict__ out_size, int32_t *__restrict__ out_val,
                                                  double *__restrict__ out_score, int32_t no_nan_exit, int32_t rbatch) {
  extern __shared__ double smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, waves = blockDim.x >> 6;
  double *hs = smem + int64_t(wave) * (topk + 1);
  int32_t *hv = reinterpret_cast<int32_t *>(smem + int64_t(waves) * (topk + 1)) + int64_t(wave) * (topk + 1);
  double *tabs = smem + int64_t(waves) * (topk + 1) + (int64_t(waves) * (topk + 1) + 1) / 2;
  double *tr12 = tabs + int64_t(wave) * 2 * kRsK, *tr2122 = tr12 + kRsK;
  const int64_t n_rows = n_rows_p[0];
  const int64_t observed = exact ? obs[1] : obs[0];
  int64_t t_next = 0, t_end = 0;
  for (;;) {
    if (t_next == t_end) {
      t_next = __shfl(lane == 0 ? int64_t(atomicAdd(row_ctr, (unsigned long long)rbatch)) : 0ll, 0, 64);
      t_end = t_next + rbatch;
    }
    const int64_t t = t_next++;
    if (t >= n_rows) break;
    const int32_t a = rows ? rows[t] : int32_t(t);
    const RowTerms R(observed, rs_row_sum(grs, a, exact));
    const int64_t n = src.size(a);
    int32_t size = 0;
    double least = 0.0;
    const int64_t rb = n > 0 ? src.base(a) : 0;
    if (lane < kRsK) {  // (the previous row's reads of them are behind its last step's wave barrier)
      tr12[lane] = xlogx(R.rs_a - lane);
      tr2122[lane] = xlogx(observed + 2 * int64_t(lane) - R.rs_a);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // the pipeline: A = the step being scored (entry, column terms), B = the next (entry; terms in flight),
    // C = the one after (entry in flight)
    int32_t cA = 0, cB = 0;
    uint32_t vA = 0u, vB = 0u;
    if (lane < n) src.get_at(rb, lane, cA, vA);
    if (64 + lane < n) src.get_at(rb, 64 + lane, cB, vB);
    ColTerms tA{};
    if (vA != 0u) tA = cterm[cA];
    for (int64_t i0 = 0; i0 < n; i0 += 64) {
      int32_t cC = 0;
      uint32_t vC = 0u;
      if (i0 + 128 + lane < n) src.get_at(rb, i0 + 128 + lane, cC, vC);
      ColTerms tB{};
      if (vB != 0u) tB = cterm[cB];
      double score = 0.0;
      if (vA != 0u) {
        const int64_t k11 = exact ? int64_t(vA) : int64_t(int16_t(uint16_t(vA)));
        if (k11 == 1) {  // ItemRowRescorer...java:203-205,230-240 (xlogx(1) = 0)
          const int64_t k22 = R.observed + k11 - (R.rs_a - k11) - (tA.rs - k11);
          score = llr_terms(R.x_all1, R.x_a, R.x_r1, tA.x_rs, tA.x_or2, 0.0, R.x_a1, tA.x_rs1, xlogx(k22));
        } else {  // LogLikelihood.java:41-57, the count-only and row-only terms from tables (as k_rescore)
          const int64_t k12 = R.rs_a - k11;
          const int64_t k21 = tA.rs - k11;
          const int64_t k22 = R.observed + k11 - k12 - k21;
          const bool in = k11 >= -32768 && k11 < 32768, inK = k11 >= 0 && k11 < kRsK;
          const double x_all = in ? k11t[k11 + 32768 + 65536] : xlogx(k11 + k12 + (k21 + k22));
          const double x_11 = in ? k11t[k11 + 32768] : xlogx(k11);
          const double x_12 = inK ? tr12[k11] : xlogx(k12);
          const double x_2122 = inK ? tr2122[k11] : xlogx(k21 + k22);
          const double x_21 = (k21 >= -32768 && k21 < 32768) ? k11t[k21 + 32768] : xlogx(k21);
          score = llr_terms(x_all, R.x_a, x_2122, tA.x_rs, xlogx(k12 + k22), x_11, x_12, x_21, xlogx(k22));
        }
      }
      const int32_t c = vA != 0u ? cA : -1;
      uint64_t m = __ballot(c >= 0 && (size < topk || score > least));
      while (m) {  // in lane order: the reference's sequential offers
        const int l = __ffsll(static_cast<unsigned long long>(m)) - 1;
        m &= m - 1;
        const double sc = __shfl(score, l, 64);
        const int32_t cl = __shfl(c, l, 64);
        if (size < topk) {
          heap_add(hv, hs, size, cl, sc);
        } else if (sc > hs[1]) {
          heap_update(hv, hs, size, cl, sc);
        }
        least = hs[1];
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // a full heap whose root is NaN takes nothing more (score > NaN is false): the rest of the row is not read
      if (!no_nan_exit && size == topk && __builtin_isnan(least)) break;
      cA = cB;
      vA = vB;
      tA = tB;
      cB = cC;
      vB = vC;
    }
    out_size[t] = size;
    for (int32_t i = lane; i < size; i += 64) {
      out_val[t * topk + i] = hv[i + 1];
      out_score[t * topk + i] = hs[i + 1];
    }
  }
}

// ---- k_rescore3: the same rescoring with every operand staged by LDS-DMA ------------------------------------
// k_rescore2's register pipeline does not survive the compiler: a gather's destination registers are reused (and
// zeroed for empty lanes) every step, so each step starts with s_waitcnt vmcnt(0) and at most one step of column
// terms is ever in flight per wave (the PMC of the full-scoring pass: ~66 requests in flight per CU, 631-cycle
// L2 latency, waves waiting 53% of their cycles).  Here a wave streams its row through a 4-slot LDS ring with
// global_load_lds (no destination register): step j is scored while the column terms of steps j + 1 and j + 2 and
// the entries of steps j + 1 .. j + 3 are in flight; counted waits (vmcnt(4), vmcnt(8): every step issues exactly 4
// DMA instructions, the clamped tail included) order the ring, and the ring is read by inline ds_reads, which the
// compiler does not pair with the DMA writes (it would otherwise wait vmcnt(0) before each).  The slow entries'
// count-only log terms come from LDS tables over k11 < 256 instead of the global k11t.  Same scores, same heaps.
constexpr int kR3Waves = 4, kR3Slots = 4, kR3L = 3, kR3G = 2, kR3K = 256;
struct R3Slot {
  uint32_t col[64];
  uint32_t cnt[64];
  uint4 lo[64];  // ColTerms bytes 0-15: rs, x_rs
  uint4 hi[64];  // ColTerms bytes 16-31: x_rs1, x_or2
};
#define R3_LDS(p) ((__attribute__((address_space(3))) void *)(p))
__device__ inline uint32_t r3_rd32(const void *p) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(uint32_t(uintptr_t(R3_LDS(p)))) : "memory");
  return v;
}
typedef uint32_t r3_u32x4 __attribute__((ext_vector_type(4)));
__device__ inline r3_u32x4 r3_rd128(const void *p) {
  r3_u32x4 v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(uint32_t(uintptr_t(R3_LDS(p)))) : "memory");
  return v;
}
template <int N>
__device__ inline void r3_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__global__ __launch_bounds__(64 * kR3Waves) void k_rescore3(
    const int32_t *__restrict__ rows, const int64_t *__restrict__ n_rows_p, CsrRows src, const int64_t *__restrict__ grs,
    const ColTerms *__restrict__ cterm, const int64_t *__restrict__ obs, int32_t exact,
    unsigned long long *__restrict__ row_ctr, int32_t topk, int32_t *__restrict__ out_size, int32_t *__restrict__ out_val,
    double *__restrict__ out_score, int32_t no_nan_exit, int32_t rbatch, int32_t exp) {
  __shared__ R3Slot ring[kR3Waves][kR3Slots];
  extern __shared__ double smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // dynamic LDS: [x11t kR3K][xallt kR3K] doubles, per wave [tr12 kRsK][tr2122 kRsK] doubles, the heaps
  double *x11t = smem, *xallt = smem + kR3K;
  double *tr12 = smem + 2 * kR3K + int64_t(wave) * 2 * kRsK, *tr2122 = tr12 + kRsK;
  double *hs = smem + 2 * kR3K + kR3Waves * 2 * kRsK + int64_t(wave) * (topk + 1);
  int32_t *hv = reinterpret_cast<int32_t *>(smem + 2 * kR3K + kR3Waves * 2 * kRsK + kR3Waves * (topk + 1)) +
                int64_t(wave) * (topk + 1);
  const int64_t n_rows = n_rows_p[0];
  const int64_t observed = exact ? obs[1] : obs[0];
  for (int k = threadIdx.x; k < kR3K; k += 64 * kR3Waves) {  // xlogx(k11) and xlogx(observed + 2 k11), k11 < 256
    x11t[k] = xlogx(k);
    xallt[k] = xlogx(observed + 2 * int64_t(k));
  }
  __syncthreads();
  R3Slot *rg = ring[wave];
  int64_t t_next = 0, t_end = 0;
  for (;;) {
    if (t_next == t_end) {
      t_next = __shfl(lane == 0 ? int64_t(atomicAdd(row_ctr, (unsigned long long)rbatch)) : 0ll, 0, 64);
      t_end = t_next + rbatch;
    }
    const int64_t t = t_next++;
    if (t >= n_rows) break;
    const int32_t a = rows ? rows[t] : int32_t(t);
    const RowTerms R(observed, rs_row_sum(grs, a, exact));
    const int64_t n = src.size(a);
    int32_t size = 0;
    double least = 0.0;
    if (n > 0) {
      const int64_t rb = src.base(a);
      if (lane < kRsK) {
        tr12[lane] = xlogx(R.rs_a - lane);
        tr2122[lane] = xlogx(observed + 2 * int64_t(lane) - R.rs_a);
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const int64_t nsteps = (n + 63) >> 6;
      for (int64_t j = -kR3L; j < nsteps; j++) {
        {  // entries of step j + L (clamped to the row's last entry past its end: every step issues 2 DMAs)
          const int64_t jl = j + kR3L;
          const int64_t e = min(jl * 64 + lane, n - 1);
          R3Slot &sl = rg[jl & (kR3Slots - 1)];
          __builtin_amdgcn_global_load_lds(src.col + rb + e, R3_LDS(sl.col), 4, 0, 0);
          __builtin_amdgcn_global_load_lds(src.cnt + rb + e, R3_LDS(sl.cnt), 4, 0, 0);
        }
        r3_wait_vm<4>();  // the entries of step j + G (issued one step ago) have landed
        {  // column terms of step j + G (outside the row: column 0's, never read)
          const int64_t jg = j + kR3G;
          R3Slot &sl = rg[jg & (kR3Slots - 1)];
          const uint32_t c = (jg >= 0 && jg < nsteps) ? r3_rd32(&sl.col[lane]) : 0u;
          const ColTerms *p = cterm + c;
          __builtin_amdgcn_global_load_lds(p, R3_LDS(sl.lo), 16, 0, 0);
          __builtin_amdgcn_global_load_lds(reinterpret_cast<const char *>(p) + 16, R3_LDS(sl.hi), 16, 0, 0);
        }
        if (j < 0) continue;
        r3_wait_vm<8>();  // the column terms of step j (issued two steps ago) have landed
        const R3Slot &sl = rg[j & (kR3Slots - 1)];
        const bool in_row = j * 64 + lane < n;
        const int32_t cA = int32_t(r3_rd32(&sl.col[lane]));
        const uint32_t vA = in_row ? r3_rd32(&sl.cnt[lane]) : 0u;
        double score = 0.0;
        if (exp == 2) {  // (timing experiment, results invalid: no scoring)
          score = vA != 0u ? double(vA) + double(cA) : 0.0;
        } else if (vA != 0u) {
          const r3_u32x4 lo = r3_rd128(&sl.lo[lane]), hi = r3_rd128(&sl.hi[lane]);
          const int64_t rs_b = int64_t((uint64_t(lo.y) << 32) | lo.x);
          const double x_rs = __longlong_as_double(int64_t((uint64_t(lo.w) << 32) | lo.z));
          const double x_rs1 = __longlong_as_double(int64_t((uint64_t(hi.y) << 32) | hi.x));
          const double x_or2 = __longlong_as_double(int64_t((uint64_t(hi.w) << 32) | hi.z));
          const int64_t k11 = exact ? int64_t(vA) : int64_t(int16_t(uint16_t(vA)));
          if (k11 == 1) {  // ItemRowRescorer...java:203-205,230-240 (xlogx(1) = 0)
            const int64_t k22 = R.observed + k11 - (R.rs_a - k11) - (rs_b - k11);
            score = llr_terms(R.x_all1, R.x_a, R.x_r1, x_rs, x_or2, 0.0, R.x_a1, x_rs1, xlogx(k22));
          } else {  // LogLikelihood.java:41-57 with the count-only and row-only terms from LDS tables
            const int64_t k12 = R.rs_a - k11;
            const int64_t k21 = rs_b - k11;
            const int64_t k22 = R.observed + k11 - k12 - k21;
            const bool inT = k11 >= 0 && k11 < kR3K, inK = k11 >= 0 && k11 < kRsK;
            const double x_all = inT ? xallt[k11] : xlogx(k11 + k12 + (k21 + k22));
            const double x_11 = inT ? x11t[k11] : xlogx(k11);
            const double x_12 = inK ? tr12[k11] : xlogx(k12);
            const double x_2122 = inK ? tr2122[k11] : xlogx(k21 + k22);
            const double x_21 = (k21 >= 0 && k21 < kR3K) ? x11t[k21] : xlogx(k21);
            score = llr_terms(x_all, R.x_a, x_2122, x_rs, xlogx(k12 + k22), x_11, x_12, x_21, xlogx(k22));
          }
        }
        const int32_t c = vA != 0u ? cA : -1;
        if (exp == 1) {  // (timing experiment, results invalid: no heap)
          if (c >= 0 && score > least) least = score;
          continue;
        }
        uint64_t m = __ballot(c >= 0 && (size < topk || score > least));
        while (m) {  // in lane order: the reference's sequential offers
          const int l = __ffsll(static_cast<unsigned long long>(m)) - 1;
          m &= m - 1;
          const double sc = __shfl(score, l, 64);
          const int32_t cl = __shfl(c, l, 64);
          if (size < topk) {
            heap_add(hv, hs, size, cl, sc);
          } else if (sc > hs[1]) {
            heap_update(hv, hs, size, cl, sc);
          }
          least = hs[1];
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (!no_nan_exit && size == topk && __builtin_isnan(least)) break;
      }
      r3_wait_vm<0>();  // (the ring's last DMAs: the next row reuses the slots)
    }
    out_size[t] = size;
    for (int32_t i = lane; i < size; i += 64) {
      out_val[t * topk + i] = hv[i + 1];
      out_score[t * topk + i] = hs[i + 1];
    }
  }
}

// ---- k_rs_score + k_rs_heap: the rescoring in two passes (owned rows against whole-log row sums) ------------------
// k_rescore3 is bound by its column-term gathers: every entry reads a 32-B ColTerms of a table (32 MB at 1e6 items)
// that no XCD's 4 MB L2 holds, so its lines come from the Infinity Cache at ~600 cycles each (the C5 owner unit's
// PMC: L2 hit 31%, waves waiting 53% of their cycles).  Here pass 1 (k_rs_score) scores the entries column block by
// column block -- kRsB blocks of the row order's columns (ascending rank_of[col], or col), block b's work queued on
// counter b % 8 in block order and taken first by the workgroups with blockIdx % 8 == b % 8 (one XCD under the
// round-robin placement; speed only, any workgroup may take any item), so at any time an XCD gathers from the terms
// of about one block (~0.5 MB) -- and writes every score's f32 upper bound (4 B) to a dense array beside the
// entries; pass 2 (k_rs_heap) streams each row's bounds in order through an LDS-DMA ring, recomputes the exact
// score of the entries whose bound beats the heap's root, and feeds those to the heap exactly as k_rescore3 does
// (the sequential loop of ItemRowRescorer...java:199-223; NaN roots end the row).  The scores are k_rescore3's bit
// for bit: the same formulas over the same integers (the row-only and count-only terms through xlogx or the k11
// tables of the same argument).  Pass 1 scores every entry (no NaN-root exit), so this is the
// path for whole-log row sums, whose heaps are numeric (the C5 owner unit: 2.7% NaN roots); k_rescore3 keeps the
// local-row-sum case, whose roots are NaN almost everywhere and whose rows end after one step.
constexpr int kRsB = 64;                                  // column blocks
// Pass 1 stores, per entry, not its score but an upper bound of it: the score rounded up to f32 (4 B).  Pass 2
// offers the heap an entry only when the bound is above the heap's root (or the heap is not full) and recomputes
// that entry's exact score then (LogLikelihood.java:41-57 over the same integers: the same bits); an entry whose
// bound is <= the root has a score <= the root and the reference would not take it (score > getLeastScore(),
// ItemRowRescorer...java:218-222).  About 1% of the entries are recomputed; 4 B per entry are written and read
// instead of 8.  A NaN score is stored as a quiet NaN (its bound compares false: recomputed); a zero count as
// kRsZero32.
constexpr uint32_t kRsZero32 = 0x7F80DEADu;               // (a signalling NaN: no rounding result has these bits)
__device__ inline uint32_t rs_bound(double sc) {
  return sc != sc ? 0x7FC00000u : __float_as_uint(__double2float_ru(sc));
}
__device__ inline int32_t rs_blk(const int32_t *__restrict__ rank_of, int32_t c, int32_t bw) {
  return min(kRsB - 1, (rank_of ? rank_of[c] : c) / bw);
}

// bp[t (kRsB + 1) + b] = the first entry of row t whose block is >= b (bp[.. + kRsB] = the row's length): one wave
// per row, lane b binary-searching bound b over the row's block ids (about log2(n) probes per bound instead of a
// rank lookup per entry)
__global__ __launch_bounds__(256) void k_rs_bounds(int64_t n_rows, CsrRows src, const int32_t *__restrict__ rank_of,
                                                   int32_t bw, int32_t *__restrict__ bp, int64_t per_q,
                                                   int32_t *__restrict__ item_len) {
  static_assert(kRsB == 64, "one bound per lane");
  const int lane = threadIdx.x & 63;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t t = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; t < n_rows; t += n_waves) {
    int32_t *o = bp + t * (kRsB + 1);
    const int32_t n = int32_t(src.size(int32_t(t)));
    int32_t lo = 0;
    if (n > 0 && lane > 0) {
      const int64_t rb = src.base(int32_t(t));
      int32_t hi = n;
      while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (rs_blk(rank_of, src.col[rb + mid], bw) < lane) lo = mid + 1; else hi = mid;
      }
    }
    o[lane] = lo;
    if (lane == 0) o[kRsB] = max(n, 0);
    // the row's share of its work items' entries (item g = (b % 8) per_q + (b / 8) n_chunks + t / 64)
    const int32_t above = __shfl_down(lo, 1, 64);  // (every lane takes part in the shuffle)
    const int32_t next = lane < 63 ? above : max(n, 0);
    if (next > lo)
      atomicAdd(item_len + int64_t(lane & 7) * per_q + int64_t(lane >> 3) * ((n_rows + 63) >> 6) + (t >> 6), next - lo);
  }
}

// The slow entries' terms that depend on a row or a column and the count only, for counts k11 < kRsTK: per row t
// trow[t][k] = {xlogx(rs_a - k) = x(k12), xlogx(observed + 2k - rs_a) = x(k21 + k22)}, per column b
// tcol[b][k] = {xlogx(observed + 2k - rs_b) = x(k12 + k22), xlogx(rs_b - k) = x(k21)} (the same integers as the
// formula's, so the same bits): a slow entry then takes one log (x(k22)) instead of four
constexpr int kRsTK = 8;
__global__ void k_rs_tables(int32_t M, const int32_t *__restrict__ row_nnz, const int64_t *__restrict__ grs,
                            const int64_t *__restrict__ obs, int32_t exact, double *__restrict__ trow,
                            double *__restrict__ tcol) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= int64_t(M) * kRsTK) return;
  const int32_t a = int32_t(i / kRsTK);
  const int64_t k = i % kRsTK;
  const int64_t observed = exact ? obs[1] : obs[0];
  const int64_t rs = rs_row_sum(grs, a, exact);
  if (row_nnz[a] > 0) {
    trow[2 * i] = xlogx(rs - k);
    trow[2 * i + 1] = xlogx(observed + 2 * k - rs);
  }
  tcol[2 * i] = xlogx(observed + 2 * k - rs);
  tcol[2 * i + 1] = xlogx(rs - k);
}

// pass 1: one wave per work item = (64 consecutive rows, one block): the item's entries, concatenated over its
// rows (a wave prefix of the rows' block lengths), are scored in rounds of 64 x kRsU, the next round's entries
// loaded while the current one's column terms are gathered and scored (a two-stage register pipeline).  Entries
// with k11 == 1 (one log) are scored in place; the others are queued in LDS with their column terms and scored 64
// at a time (one log each with the row / column tables), so that no wave runs both paths for a few lanes.
#ifndef COOC_RS_U
#define COOC_RS_U 2  // (A/B builds: scripts/build_variant.sh)
#endif
constexpr int kRsU = COOC_RS_U;
#ifndef COOC_RS_GRAB
#define COOC_RS_GRAB 8  // (A/B builds)
#endif
constexpr int kRsGrab = COOC_RS_GRAB;  // work units per counter grab
constexpr int kRsQ = 128;  // queue capacity: < 64 left over + one sub-round's 64
constexpr int kRsXT = 256; // LDS tables of x(k11) and x(observed + 2 k11), k11 < kRsXT
struct RsItem {
  int64_t t0;        // the item's first row
  int32_t off[65];   // exclusive prefix of the rows' block lengths (off[64] = the item's entries)
  int64_t src[64];   // a row's first entry of the block in the CSR arena
  int64_t dst[64];   // ... and its score slot
  int64_t rs[64];    // the row's sum
  double rt[64][4];  // RowTerms: x_a, x_all1, x_r1, x_a1
  int32_t qk[kRsQ];  // queued entries: item-relative index, count, column's row sum and x(rs_b), column
  uint32_t qv[kRsQ];
  int64_t qrs[kRsQ];
  double qxrs[kRsQ];
  int32_t qc[kRsQ];
};
__device__ inline int rs_item_row(const RsItem &it, int32_t k) {
  int r = 0;
#pragma unroll
  for (int st = 32; st > 0; st >>= 1)
    if (it.off[r + st] <= k) r += st;
  return r;
}
// the full formula (LogLikelihood.java:41-57) for queue slot j (lanes past the queue: l >= n)
__device__ inline void rs_score_slow(const RsItem &it, int j, bool on, const double *xt,
                                     const double *__restrict__ k11t, const double *__restrict__ trow,
                                     const double *__restrict__ tcol, int64_t observed, int32_t exact,
                                     uint32_t *__restrict__ score, int32_t *__restrict__ nanrow) {
#pragma clang fp contract(off)
  if (!on) return;
  const int32_t k = it.qk[j];
  const uint32_t v = it.qv[j];
  const int64_t rs_b = it.qrs[j];
  const int32_t c = it.qc[j];
  const int r = rs_item_row(it, k);
  const int64_t k11 = exact ? int64_t(v) : int64_t(int16_t(uint16_t(v)));
  const int64_t rs_a = it.rs[r];
  const int64_t k12 = rs_a - k11;
  const int64_t k21 = rs_b - k11;
  const int64_t k22 = observed + k11 - k12 - k21;
  const bool inX = k11 >= 0 && k11 < kRsXT;
  const bool in = k11 >= -32768 && k11 < 32768;
  const double x_all = inX ? xt[kRsXT + k11] : in ? k11t[k11 + 32768 + 65536] : xlogx(k11 + k12 + (k21 + k22));
  const double x_11 = inX ? xt[k11] : in ? k11t[k11 + 32768] : xlogx(k11);
  const bool inT = k11 >= 0 && k11 < kRsTK;
  double x_12, x_2122, x_1222, x_21;
  if (inT) {
    const double *tr = trow + ((it.t0 + r) * kRsTK + k11) * 2;
    const double *tc = tcol + (int64_t(c) * kRsTK + k11) * 2;
    x_12 = tr[0];
    x_2122 = tr[1];
    x_1222 = tc[0];
    x_21 = tc[1];
  } else {
    x_12 = xlogx(k12);
    x_2122 = xlogx(k21 + k22);
    x_1222 = xlogx(k12 + k22);
    x_21 = (k21 >= -32768 && k21 < 32768) ? k11t[k21 + 32768] : xlogx(k21);
  }
  const double sc = llr_terms(x_all, it.rt[r][0], x_2122, it.qxrs[j], x_1222, x_11, x_12, x_21, xlogx(k22));
  if (sc != sc) nanrow[it.t0 + r] = 1;
  score[it.dst[r] + (k - it.off[r])] = rs_bound(sc);
}
// Work units of pass 1: the items (64 consecutive rows x one block; queue q = block % 8 holds its blocks' items in
// block order, so item g = q per_q + (b / 8) n_chunks + chunk) cut into pieces of at most kRsP entries, so that
// no wave is left alone with the hot rows' items (the Zipf head: ~1e5 entries per item).  units[g] = the item's
// pieces (item_len[g]: the item's entries, summed by k_rs_bounds; item_len[n] = 0, so ubase[n], the exclusive
// prefix of the pieces, is the total); umap[u] = the item of unit u.
#ifndef COOC_RS_P
#define COOC_RS_P 4096  // (A/B builds)
#endif
constexpr int32_t kRsP = COOC_RS_P;
struct ScanUnits {  // the pieces of item g, from its entry count (k_rs_bounds)
  const int32_t *len;
  __device__ int64_t operator()(int64_t g) const { return (int64_t(len[g]) + kRsP - 1) / kRsP; }
};
__global__ void k_rs_unit_map(int64_t n, const int32_t *__restrict__ item_len, const int64_t *__restrict__ ubase,
                              int32_t *__restrict__ umap) {
  const int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const int64_t np = ScanUnits{item_len}(g);
  for (int64_t p = 0; p < np; p++) umap[ubase[g] + p] = int32_t(g);
}

__global__ __launch_bounds__(256) void k_rs_score(int64_t n_rows, CsrRows src, const int32_t *__restrict__ bp,
                                                  const int64_t *__restrict__ sbase, const int64_t *__restrict__ grs,
                                                  const ColTerms *__restrict__ cterm, const double *__restrict__ k11t,
                                                  const double *__restrict__ trow, const double *__restrict__ tcol,
                                                  const int64_t *__restrict__ obs, int32_t exact,
                                                  const int64_t *__restrict__ ubase, const int32_t *__restrict__ umap,
                                                  unsigned long long *__restrict__ qctr, uint32_t *__restrict__ score,
                                                  int32_t *__restrict__ nanrow, int32_t exp) {
#pragma clang fp contract(off)
  __shared__ RsItem items[4];
  __shared__ double xt[2 * kRsXT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const int64_t n_chunks = (n_rows + 63) >> 6;
  const int64_t per_q = n_chunks * (kRsB / 8);
  const int64_t observed = exact ? obs[1] : obs[0];
  for (int k = threadIdx.x; k < kRsXT; k += 256) {
    xt[k] = k11t[k + 32768];
    xt[kRsXT + k] = k11t[k + 32768 + 65536];
  }
  __syncthreads();
  RsItem &it = items[wave];
  const int q0 = int(blockIdx.x & 7);
  for (int qi = 0; qi < 8; qi++) {
    const int q = (q0 + qi) & 7;
    const int64_t u_lo = ubase[q * per_q], n_units = ubase[(q + 1) * per_q] - u_lo;
    int64_t j_next = 0, j_end = 0;
    for (;;) {
      if (j_next == j_end) {  // kRsGrab units per counter grab (one counter serves a quarter of the chip's waves)
        j_next = __shfl(lane == 0 ? int64_t(atomicAdd(qctr + q, (unsigned long long)kRsGrab)) : 0ll, 0, 64);
        j_end = min(j_next + kRsGrab, n_units);
      }
      if (j_next >= n_units) break;
      const int64_t u = u_lo + j_next++;
      const int64_t g = umap[u];
      const int32_t kb = int32_t(u - ubase[g]) * kRsP;  // the unit's piece of the item
      const int64_t item = g - q * per_q;
      const int b = q + 8 * int(item / n_chunks);
      const int64_t t = ((item % n_chunks) << 6) + lane;
      int32_t e0 = 0, len = 0;
      if (t < n_rows) {
        e0 = bp[t * (kRsB + 1) + b];
        len = bp[t * (kRsB + 1) + b + 1] - e0;
      }
      int32_t incl = len;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int32_t v = __shfl_up(incl, d, 64);
        if (lane >= d) incl += v;
      }
      const int32_t T = __shfl(incl, 63, 64);
      if (T == 0) continue;
      it.off[lane] = incl - len;
      if (lane == 63) it.off[64] = T;
      if (lane == 0) it.t0 = t;
      if (len > 0) {
        const int32_t a = int32_t(t);
        const int64_t rs_a = rs_row_sum(grs, a, exact);
        // RowTerms from the tables (the same xlogx of the same integers): x(rs_a) = trow[a][0].x, x(rs_a - 1) =
        // trow[a][1].x, x(observed + 2 - rs_a) = trow[a][1].y, x(observed + 2) = the k11 table at k11 = 1
        const double *tr = trow + int64_t(a) * kRsTK * 2;
        it.src[lane] = src.base(a) + e0;
        it.dst[lane] = sbase[t] + e0;
        it.rs[lane] = rs_a;
        it.rt[lane][0] = tr[0];
        it.rt[lane][1] = k11t[1 + 32768 + 65536];
        it.rt[lane][2] = tr[3];
        it.rt[lane][3] = tr[2];
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (exp & 32) continue;  // (timing experiment: the items' overhead alone)
      const int32_t ke = min(T, kb + kRsP);
      int32_t nq = 0;  // queued entries (wave-uniform)
      int32_t cA[kRsU], rA[kRsU];
      uint32_t vA[kRsU];
#pragma unroll
      for (int u = 0; u < kRsU; u++) {  // round 0's entries
        const int32_t k = kb + u * 64 + lane;
        const int r = rs_item_row(it, k);
        rA[u] = r;
        cA[u] = 0;
        vA[u] = 0u;
        if (k < ke) {
          cA[u] = src.col[it.src[r] + (k - it.off[r])];
          vA[u] = src.cnt[it.src[r] + (k - it.off[r])];
        }
      }
      for (int32_t k0 = kb; k0 < ke; k0 += 64 * kRsU) {
        ColTerms h[kRsU];
#pragma unroll
        for (int u = 0; u < kRsU; u++)  // the current round's column terms
          if (k0 + u * 64 + lane < ke && vA[u] != 0u) h[u] = (exp & 4) ? ColTerms{cA[u], 1.0, 2.0, 3.0} : cterm[cA[u]];
        int32_t cB[kRsU], rB[kRsU];
        uint32_t vB[kRsU];
#pragma unroll
        for (int u = 0; u < kRsU; u++) {  // the next round's entries (the row of entry k: the last with off <= k)
          const int32_t k = k0 + (kRsU + u) * 64 + lane;
          cB[u] = 0;
          vB[u] = 0u;
          rB[u] = 0;
          if (k < ke) {
            const int r = rs_item_row(it, k);
            rB[u] = r;
            cB[u] = src.col[it.src[r] + (k - it.off[r])];
            vB[u] = src.cnt[it.src[r] + (k - it.off[r])];
          }
        }
#pragma unroll
        for (int u = 0; u < kRsU; u++) {
          const int32_t k = k0 + u * 64 + lane;
          const int r = rA[u];  // (found when the entry was loaded)
          const int64_t k11 = exact ? int64_t(vA[u]) : int64_t(int16_t(uint16_t(vA[u])));
          const bool valid = k < ke;
          const bool slow = valid && vA[u] != 0u && k11 != 1;
          if (valid && !slow) {
            uint32_t bits = kRsZero32;
            if (vA[u] != 0u) {  // ItemRowRescorer...java:203-205,230-240 (xlogx(1) = 0)
              const int64_t rs_a = it.rs[r];
              const int64_t k22 = observed + k11 - (rs_a - k11) - (h[u].rs - k11);
              const double sc = llr_terms(it.rt[r][1], it.rt[r][0], it.rt[r][2], h[u].x_rs, h[u].x_or2, 0.0,
                                          it.rt[r][3], h[u].x_rs1, (exp & 2) ? double(k22) : xlogx(k22));
              if (sc != sc) nanrow[it.t0 + r] = 1;  // (a NaN score: the row's heap pass cannot be split, k_rs_heap)
              bits = rs_bound(sc);
            }
            if (!(exp & 8) || bits == 0x1234u) score[it.dst[r] + (k - it.off[r])] = bits;
          }
          const uint64_t sm = __ballot(slow);
          if (slow) {
            const int j = nq + int32_t(__popcll(sm & lt));
            it.qk[j] = k;
            it.qv[j] = vA[u];
            it.qrs[j] = h[u].rs;
            it.qxrs[j] = h[u].x_rs;
            it.qc[j] = cA[u];
          }
          nq += int32_t(__popcll(sm));
          if (exp & 1) nq = 0;  // (timing experiments, results invalid: 1 no slow entries, 2 no fast-path log,
                                //  4 no gather, 8 no store)
          if (nq >= 64) {       // a full batch of queued entries
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            nq -= 64;
            rs_score_slow(it, nq + lane, true, xt, k11t, trow, tcol, observed, exact, score, nanrow);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
          }
        }
#pragma unroll
        for (int u = 0; u < kRsU; u++) {
          cA[u] = cB[u];
          vA[u] = vB[u];
          rA[u] = rB[u];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      rs_score_slow(it, lane, lane < nq, xt, k11t, trow, tcol, observed, exact, score, nanrow);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// pass 2: one wave per row, its columns and scores streamed through a kR5Slots-slot LDS-DMA ring (3 DMAs per step of
// 64 entries, issued kR5L steps ahead, 9 KB in flight per wave: the Zipf head's rows of ~1e6 entries run on one wave
// each; counted waits as in k_rescore3), the heap fed in column order
#ifndef COOC_R5_SLOTS
#define COOC_R5_SLOTS 16  // (A/B builds; 8 slots / 6 ahead: 13.0 ms on the owner unit, 16 / 10-14: 11.8)
#define COOC_R5_L 12
#endif
#ifndef COOC_R5_WAVES
#define COOC_R5_WAVES 4
#endif
constexpr int kR5Waves = COOC_R5_WAVES, kR5Slots = COOC_R5_SLOTS, kR5L = COOC_R5_L;
struct R5Slot {  // a step's score bounds (the heap holds entry indices: the columns are read for the k kept, at the end)
  uint32_t ub[64];
};
// Rows longer than kRsLong entries whose scores hold no NaN are cut into segments of kRsSeg entries, one wave each:
// a segment feeds a heap of its own from empty and keeps, in order, every entry that heap could take (at most
// kRsCand; more: the row is replayed whole).  An entry a full segment heap refuses (score <= its root) is refused by
// the row's heap too, whose root is the k-th largest score of a superset of the entries before it (a total order:
// no NaN); refused entries change nothing, so the row's heap fed only the kept entries, in order, ends exactly as
// fed every entry.  The wave that finishes a row's last segment replays the kept entries into the row's heap.
constexpr int64_t kRsLong = 65536;
constexpr int32_t kRsSeg = 16384, kRsCand = 2048;
__global__ void k_rs_seg_count(int64_t n_rows, CsrRows src, const int32_t *__restrict__ nanrow, int64_t long_thr,
                               int32_t seg_len, int32_t *__restrict__ nseg) {
  const int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t > n_rows) return;
  if (t == n_rows) {
    nseg[t] = 0;
    return;
  }
  const int64_t n = src.size(int32_t(t));
  nseg[t] = (n > long_thr && !nanrow[t]) ? int32_t((n + seg_len - 1) / seg_len) : 0;
}

// The exact score of entry i of row a (pass 2's recomputation): LogLikelihood.java:41-57 over k11 (the entry's
// count or its int16 view), k12 = rs_a - k11, k21 = rs_b - k11, k22 = observed + k11 - k12 - k21
// (ItemRowRescorer...java:230-240) -- the integers pass 1 used, so the same bits.
struct RsExact {
  const int64_t *grs;
  int64_t observed;
  int32_t exact;
  __device__ double operator()(CsrRows src, int64_t rb, int64_t i, int64_t rs_a) const {
#pragma clang fp contract(off)
    const int32_t c = src.col[rb + i];
    const uint32_t v = src.cnt[rb + i];
    const int64_t k11 = exact ? int64_t(v) : int64_t(int16_t(uint16_t(v)));
    const int64_t rs_b = rs_row_sum(grs, c, exact);
    const int64_t k12 = rs_a - k11, k21 = rs_b - k11;
    return llr(k11, k12, k21, observed + k11 - k12 - k21);
  }
};

// Feeds one step's offers (lanes with c >= 0, exact scores sc) to the heap in lane order; returns the offer mask.
__device__ inline uint64_t rs_feed(bool cand, int32_t c, double sc, int32_t topk, int32_t *hv, double *hs,
                                   int32_t &size, double &least) {
  const uint64_t m0 = __ballot(cand && (size < topk || sc > least));
  uint64_t m = m0;
  while (m) {  // in lane order: the reference's sequential offers
    const int l = __ffsll(static_cast<unsigned long long>(m)) - 1;
    m &= m - 1;
    const double s_l = __shfl(sc, l, 64);
    const int32_t c_l = __shfl(c, l, 64);
    if (size < topk) {
      heap_add(hv, hs, size, c_l, s_l);
    } else if (s_l > hs[1]) {
      heap_update(hv, hs, size, c_l, s_l);
    }
    least = hs[1];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  return m0;
}

// Streams entries [i0, i1) of a row's score bounds through the wave's ring into its heap (hv, hs, size, least);
// kSeg: also records the entries offered (a superset of those taken) as segment-relative u16 indices in
// cand[0, cand_cap), *nc counting them all.
template <bool kSeg>
__device__ inline void rs_stream(R5Slot *rg, int32_t *qb, CsrRows src, const uint32_t *__restrict__ score, RsExact ex,
                                 int64_t rs_a, int64_t rb, int64_t sb, int64_t i0, int64_t i1, int32_t topk,
                                 int32_t *hv, double *hs, int32_t &size, double &least, int32_t no_nan_exit,
                                 uint16_t *__restrict__ cand, int32_t cand_cap, int32_t &nc) {
  const int lane = threadIdx.x & 63;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const int64_t n = i1 - i0;
  const int64_t nsteps = (n + 63) >> 6;
  // Entries whose bound beats the root (as of the last feed: a superset of the offers) queue in qb in order; 64 at
  // a time they are rescored exactly (full lanes, one drain of the ring per 64 instead of per step) and fed.
  int32_t nq = 0;
  auto flush = [&](int32_t cnt) {
    const bool on = lane < cnt;
    const int32_t ii = on ? qb[lane] : 0;
    const double sc = on ? ex(src, rb, ii, rs_a) : 0.0;
    const uint64_t m = rs_feed(on, ii, sc, topk, hv, hs, size, least);
    if (kSeg) {
      if ((m >> lane) & 1ull) {
        const int32_t q = nc + int32_t(__popcll(m & lt));
        if (q < cand_cap) cand[q] = uint16_t(ii - i0);
      }
      nc += int32_t(__popcll(m));
    }
  };
  for (int64_t j = -kR5L; j < nsteps; j++) {
    {  // step j + L (clamped to the range's last entry past its end: every step issues 1 DMA)
      const int64_t jl = j + kR5L;
      const int64_t e = i0 + min(jl * 64 + lane, n - 1);
      __builtin_amdgcn_global_load_lds(score + sb + e, R3_LDS(rg[jl & (kR5Slots - 1)].ub), 4, 0, 0);
    }
    if (j < 0) continue;
    r3_wait_vm<kR5L>();  // step j's DMA (issued L steps ago) has landed
    const int64_t i = i0 + j * 64 + lane;
    const uint32_t ub = j * 64 + lane < n ? r3_rd32(&rg[j & (kR5Slots - 1)].ub[lane]) : kRsZero32;
    // a possible offer only if the bound is above the root (or the heap is not full)
    const bool offer = ub != kRsZero32 && (size < topk || !(double(__uint_as_float(ub)) <= least));
    const uint64_t b = __ballot(offer);
    if (offer) qb[nq + int32_t(__popcll(b & lt))] = int32_t(i);
    nq += int32_t(__popcll(b));
    if (nq >= 64) {
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      flush(64);
      const int32_t rest = lane + 64 < nq ? qb[lane + 64] : 0;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (lane + 64 < nq) qb[lane] = rest;
      nq -= 64;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // (a full heap with a NaN root takes nothing more: the queued entries after it would be refused too)
      if (!no_nan_exit && size == topk && __builtin_isnan(least)) break;
    }
  }
  r3_wait_vm<0>();  // (the ring's last DMAs: the next range reuses the slots)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (nq > 0 && !(!no_nan_exit && size == topk && __builtin_isnan(least))) flush(nq);
}

// pass 2: units [0, n_seg) are the long rows' segments, then one unit per row (a long row's own unit is skipped);
// one wave per unit, units taken 4 at a time.  A row streams its score bounds through a kR5Slots-slot LDS-DMA ring
// (one DMA per step of 64 entries issued kR5L steps ahead; counted waits as in k_rescore3) into the heap in column
// order (the sequential loop of ItemRowRescorer...java:199-223), ending at a full heap with a NaN root.  The heap
// orders by score alone (IntDoublePriorityQueue.java:132-205), so it holds entry indices and the k kept columns
// are read at the end.
__global__ __launch_bounds__(64 * kR5Waves) void k_rs_heap(int64_t n_rows, CsrRows src,
                                                          const int64_t *__restrict__ sbase,
                                                          const uint32_t *__restrict__ score,
                                                          const int64_t *__restrict__ grs,
                                                          const int64_t *__restrict__ obs, int32_t exact,
                                                          unsigned long long *__restrict__ row_ctr, int32_t topk,
                                                          int32_t *__restrict__ out_size, int32_t *__restrict__ out_val,
                                                          double *__restrict__ out_score, int32_t no_nan_exit,
                                                          int64_t exp_skip, const int64_t *__restrict__ segp,
                                                          uint16_t *__restrict__ cand, int32_t *__restrict__ ncand,
                                                          int32_t *__restrict__ segdone, int32_t seg_len,
                                                          int32_t cand_cap) {
  __shared__ R5Slot ring[kR5Waves][kR5Slots];
  __shared__ int32_t qbuf[kR5Waves][128];
  extern __shared__ double smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double *hs = smem + int64_t(wave) * (topk + 1);
  int32_t *hv = reinterpret_cast<int32_t *>(smem + kR5Waves * (topk + 1)) + int64_t(wave) * (topk + 1);
  R5Slot *rg = ring[wave];
  int32_t *qb = qbuf[wave];
  const RsExact ex{grs, exact ? obs[1] : obs[0], exact};
  const int64_t n_seg = segp[n_rows], n_units = n_seg + n_rows;
  int64_t u_next = 0, u_end = 0;
  for (;;) {
    if (u_next == u_end) {
      u_next = __shfl(lane == 0 ? int64_t(atomicAdd(row_ctr, 4ull)) : 0ll, 0, 64);
      u_end = u_next + 4;
    }
    const int64_t u = u_next++;
    if (u >= n_units) break;
    int32_t size = 0, nc = 0;
    double least = 0.0;
    int64_t t;
    if (u < n_seg) {  // a segment: its own heap, its offered entries kept
      int64_t lo = 0, hi = n_rows;  // t: the last row with segp[t] <= u
      while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (segp[mid] <= u) lo = mid; else hi = mid;
      }
      t = lo;
      const int64_t n = src.size(int32_t(t)), rb = src.base(int32_t(t)), sb = sbase[t];
      const int64_t rs_a = rs_row_sum(ex.grs, int32_t(t), ex.exact);
      const int64_t s0 = segp[t], ns = segp[t + 1] - s0, i0 = (u - s0) * seg_len;
      rs_stream<true>(rg, qb, src, score, ex, rs_a, rb, sb, i0, min(n, i0 + seg_len), topk, hv, hs, size, least, 1,
                      cand + u * kRsCand, cand_cap, nc);
      if (lane == 0) ncand[u] = nc;
      __threadfence();  // (the kept entries and their count, before the row's segment count)
      const int32_t done = __shfl(lane == 0 ? atomicAdd(segdone + t, 1) : 0, 0, 64);
      if (done != ns - 1) continue;
      __threadfence();  // the last segment of the row: every segment's kept entries are visible
      size = 0;
      least = 0.0;
      bool whole = false;
      for (int64_t q = 0; q < ns; q++) whole |= ncand[s0 + q] > cand_cap;
      if (whole) {
        rs_stream<false>(rg, qb, src, score, ex, rs_a, rb, sb, 0, n, topk, hv, hs, size, least, no_nan_exit, nullptr, 0,
                         nc);
      } else {
        for (int64_t q = 0; q < ns; q++) {
          const int32_t cq = ncand[s0 + q];
          for (int32_t j0 = 0; j0 < cq; j0 += 64) {
            const bool on = j0 + lane < cq;
            const int64_t i = on ? q * seg_len + cand[(s0 + q) * kRsCand + j0 + lane] : 0;
            const double sc = on ? ex(src, rb, i, rs_a) : 0.0;
            rs_feed(on, int32_t(i), sc, topk, hv, hs, size, least);
          }
        }
      }
    } else {  // a row
      t = u - n_seg;
      const int64_t n0 = src.size(int32_t(t));
      if (segp[t + 1] > segp[t]) continue;  // (its segments serve it)
      const int64_t n = (exp_skip > 0 && n0 > exp_skip) ? 0 : n0;  // (timing experiment)
      if (n > 0)
        rs_stream<false>(rg, qb, src, score, ex, rs_row_sum(ex.grs, int32_t(t), ex.exact), src.base(int32_t(t)), sbase[t],
                         0, n, topk, hv, hs, size, least, no_nan_exit, nullptr, 0, nc);
    }
    out_size[t] = size;
    if (size > 0) {
      const int64_t rb = src.base(int32_t(t));
      for (int32_t i = lane; i < size; i += 64) {
        out_val[t * topk + i] = src.col[rb + hv[i + 1]];
        out_score[t * topk + i] = hs[i + 1];
      }
    }
  }
}

size_t rescore3_lds_bytes(int32_t topk) {
  return sizeof(double) * (2 * kR3K + kR3Waves * 2 * kRsK + kR3Waves * size_t(topk + 1) +
                           (kR3Waves * size_t(topk + 1) + 1) / 2);
}

// The rescorer's observed total after one window from an empty state: sum of the int views of the
// row-sum updates (ItemRowRescorer...java:154), and the exact total (out3 zeroed by the caller).
__global__ void k_observed(const int64_t *__restrict__ rowsum, int32_t M, int64_t *__restrict__ out3) {
  __shared__ int64_t sr[4], se[4];
  int64_t r = 0, e = 0;
  for (int32_t a = blockIdx.x * 256 + threadIdx.x; a < M; a += gridDim.x * 256) {
    r += int64_t(int32_t(uint32_t(uint64_t(rowsum[a]))));
    e += rowsum[a];
  }
  for (int o = 32; o > 0; o >>= 1) {
    r += __shfl_xor(r, o, 64);
    e += __shfl_xor(e, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    sr[threadIdx.x >> 6] = r;
    se[threadIdx.x >> 6] = e;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(reinterpret_cast<unsigned long long *>(out3), (unsigned long long)(sr[0] + sr[1] + sr[2] + sr[3]));
    atomicAdd(reinterpret_cast<unsigned long long *>(out3 + 1), (unsigned long long)(se[0] + se[1] + se[2] + se[3]));
    if (blockIdx.x == 0) out3[2] = M;
  }
}

// ---- sparse global rows (n_items >= 40,320): the rescorer's itemRows (ItemRowRescorer...java:35,
// 171-177) as one sorted slab per row, g_len[a] (column, count) entries at g_base[a] of an arena.  A
// window's packed delta rows (drp, dcol, dcnt; ascending columns) are merged into a new slab per
// touched row: a delta entry whose column is new takes a slot, one whose column exists adds to it.
__device__ inline int64_t lower_bound_col(const int32_t *__restrict__ c, int64_t n, int32_t x) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (c[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// The row of packed delta entry e: the last a with drp[a] <= e (drp ascending, drp[M] = nnz).
__device__ inline int32_t gs_row_of(const int64_t *__restrict__ drp, int32_t M, int64_t e) {
  int32_t lo = 0, hi = M;  // invariant: drp[lo] <= e < drp[hi]
  while (hi - lo > 1) {
    const int32_t mid = (lo + hi) >> 1;
    if (drp[mid] <= e) lo = mid; else hi = mid;
  }
  return lo;
}

// Per delta entry (flat over the window's entries, whatever the row lengths): its column's position
// in the row's old slab (opos) and flag[e] = 1 when the column is new to the row.
__global__ __launch_bounds__(256) void k_gs_flags(int32_t M, int64_t nnz, const int64_t *__restrict__ drp,
                                                  const int32_t *__restrict__ dcol, const int64_t *__restrict__ gbase,
                                                  const int32_t *__restrict__ glen, const int32_t *__restrict__ gcol,
                                                  int32_t *__restrict__ flag, int64_t *__restrict__ opos) {
  const int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  const int32_t a = gs_row_of(drp, M, e);
  const int32_t *old = gcol + gbase[a];
  const int64_t n_old = glen[a], c = dcol[e];
  const int64_t p = lower_bound_col(old, n_old, int32_t(c));
  opos[e] = p;
  flag[e] = (p < n_old && old[p] == c) ? 0 : 1;
}

// new slab of every touched row with new columns: old + new entries, bump-allocated; a row without new
// columns keeps its slab (-2: counts added in place); chunks[a] = its old entries in kGsChunk pieces
constexpr int64_t kGsChunk = 2048;
__global__ void k_gs_alloc(int32_t M, const int64_t *__restrict__ drp, const int64_t *__restrict__ newpre,
                           const int32_t *__restrict__ glen, int64_t *__restrict__ nbase,
                           unsigned long long *__restrict__ bump, int32_t *__restrict__ chunks) {
  const int32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= M) return;
  const int64_t d0 = drp[a], d1 = drp[a + 1];
  chunks[a] = 0;
  if (d0 == d1) {
    nbase[a] = -1;
    return;
  }
  const int64_t added = newpre[d1] - newpre[d0];
  if (added == 0) {  // no new column: the counts are added in place (the slab stays)
    nbase[a] = -2;
    return;
  }
  const int64_t need = int64_t(glen[a]) + added;
  nbase[a] = int64_t(atomicAdd(bump, (unsigned long long)need));
  chunks[a] = int32_t((glen[a] + kGsChunk - 1) / kGsChunk);
}

// The moved rows' old entries, kGsChunk per block (flat over the rows, so a long row is spread over
// many blocks): an old entry shifts right by the new columns below it and takes a matching delta's count.
__global__ __launch_bounds__(256) void k_gs_move_all(int32_t M, const int64_t *__restrict__ chunk_pre,
                                                 const int64_t *__restrict__ drp, const int32_t *__restrict__ dcol,
                                                 const uint32_t *__restrict__ dcnt, const int64_t *__restrict__ newpre,
                                                 const int64_t *__restrict__ nbase, const int64_t *__restrict__ gbase,
                                                 const int32_t *__restrict__ glen, int32_t *__restrict__ gcol,
                                                 uint32_t *__restrict__ gcnt) {
  const int64_t n_chunks = chunk_pre[M];
  for (int64_t ch = blockIdx.x; ch < n_chunks; ch += gridDim.x) {
    int32_t lo = 0, hi = M;  // the row: last a with chunk_pre[a] <= ch
    while (hi - lo > 1) {
      const int32_t mid = (lo + hi) >> 1;
      if (chunk_pre[mid] <= ch) lo = mid; else hi = mid;
    }
    const int32_t a = lo;
    const int64_t i0 = (ch - chunk_pre[a]) * kGsChunk, n_old = glen[a], i1 = min(n_old, i0 + kGsChunk);
    const int64_t nb = nbase[a], d0 = drp[a], d = drp[a + 1] - d0, ob = gbase[a];
    for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
      const int32_t c = gcol[ob + i];
      const int64_t p = lower_bound_col(dcol + d0, d, c);
      const uint32_t add = (p < d && dcol[d0 + p] == c) ? dcnt[d0 + p] : 0u;
      const int64_t pos = nb + i + (newpre[d0 + p] - newpre[d0]);
      gcol[pos] = c;
      gcnt[pos] = gcnt[ob + i] + add;
    }
  }
}

// Per delta entry: a new column lands after the old columns below it in the row's new slab; in a row
// without new columns the count is added where the column sits.
__global__ __launch_bounds__(256) void k_gs_insert(int32_t M, int64_t nnz, const int64_t *__restrict__ drp,
                                                   const int32_t *__restrict__ dcol, const uint32_t *__restrict__ dcnt,
                                                   const int64_t *__restrict__ newpre, const int32_t *__restrict__ flag,
                                                   const int64_t *__restrict__ opos, const int64_t *__restrict__ nbase,
                                                   const int64_t *__restrict__ gbase, int32_t *__restrict__ gcol,
                                                   uint32_t *__restrict__ gcnt) {
  const int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  const int32_t a = gs_row_of(drp, M, e);
  const int64_t nb = nbase[a];
  if (nb == -2) {
    gcnt[gbase[a] + opos[e]] += dcnt[e];
  } else if (flag[e]) {
    const int64_t pos = nb + (newpre[e] - newpre[drp[a]]) + opos[e];
    gcol[pos] = dcol[e];
    gcnt[pos] = dcnt[e];
  }
}

__global__ void k_gs_commit(int32_t M, const int64_t *__restrict__ drp, const int64_t *__restrict__ newpre,
                            const int64_t *__restrict__ nbase, int64_t *__restrict__ gbase, int32_t *__restrict__ glen) {
  const int32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= M || nbase[a] < 0) return;
  glen[a] += int32_t(newpre[drp[a + 1]] - newpre[drp[a]]);
  gbase[a] = nbase[a];
}

// compaction: every row's slab to a fresh arena at the prefix of the row lengths (one wave per row)
__global__ __launch_bounds__(256) void k_gs_compact(int32_t M, const int64_t *__restrict__ newbase,
                                                    int64_t *__restrict__ gbase, const int32_t *__restrict__ glen,
                                                    const int32_t *__restrict__ col_in, const uint32_t *__restrict__ cnt_in,
                                                    int32_t *__restrict__ col_out, uint32_t *__restrict__ cnt_out) {
  const int lane = threadIdx.x & 63;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t a = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; a < M; a += n_waves) {
    const int64_t from = gbase[a], to = newbase[a], n = glen[a];
    for (int64_t i = lane; i < n; i += 64) {
      col_out[to + i] = col_in[from + i];
      cnt_out[to + i] = cnt_in[from + i];
    }
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) gbase[a] = to;
  }
}

struct WidenLen {
  __host__ __device__ int64_t operator()(int32_t v) const { return int64_t(v); }
};

}  // namespace
namespace {
__global__ void k_llr(int64_t n, const int64_t *__restrict__ k, double *__restrict__ out) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) out[i] = llr(k[4 * i], k[4 * i + 1], k[4 * i + 2], k[4 * i + 3]);
}
}  // namespace

Status launch_llr(hipStream_t s, int64_t n, const int64_t *d_k4, double *d_out) {
  if (n <= 0) return Status::Ok();
  k_llr<<<unsigned((n + 255) / 256), 256, 0, s>>>(n, d_k4, d_out);
  COOC_HIP_TRY(hipGetLastError());
  return Status::Ok();
}

Status launch_relocate(hipStream_t s, int64_t n, const int64_t *reloc, int32_t *arena) {
  if (n > 0) k_relocate<<<std::min<unsigned>(blocks_for(n * 64, 256), 4096), 256, 0, s>>>(n, reloc, arena);
  COOC_HIP_TRY(hipGetLastError());
  return Status::Ok();
}

Status launch_gather_lists(hipStream_t s, int64_t n, const int64_t *off, const int32_t *len, const int64_t *dst,
                           const int32_t *arena, int32_t *out) {
  if (n > 0) k_gather_lists<<<std::min<unsigned>(blocks_for(n * 64, 256), 4096), 256, 0, s>>>(n, off, len, dst, arena, out);
  COOC_HIP_TRY(hipGetLastError());
  return Status::Ok();
}

Status launch_append(hipStream_t s, int64_t n, const int64_t *new_ptr, const int64_t *new_dst, const int32_t *items,
                     int32_t *arena) {
  if (n > 0) k_append<<<std::min<unsigned>(blocks_for(n * 64, 256), 4096), 256, 0, s>>>(n, new_ptr, new_dst, items, arena);
  COOC_HIP_TRY(hipGetLastError());
  return Status::Ok();
}

Status launch_merge_global(hipStream_t s, int32_t M, const int64_t *row_base, const int32_t *row_nnz,
                           const int32_t *col, const uint32_t *cnt, const int64_t *rowsum_delta, uint32_t *G,
                           int64_t *grs, int64_t *scal, int64_t observed_window) {
  COOC_HIP_TRY(hipMemsetAsync(scal + 1, 0, sizeof(int64_t), s));
  k_merge_global<<<std::min<unsigned>(blocks_for(int64_t(M) * 64, 256), 8192), 256, 0, s>>>(
      M, row_base, row_nnz, col, cnt, rowsum_delta, G, grs, scal);
  k_finish_scalars<<<1, 1, 0, s>>>(scal, observed_window);
  COOC_HIP_TRY(hipGetLastError());
  return Status::Ok();
}

Status launch_owned_view(hipStream_t s, int32_t M, int32_t W, int32_t part, int32_t R, const int64_t *mbase,
                         const int32_t *mnnz, int64_t *base, int32_t *nnz) {
  COOC_HIP_TRY(hipMemsetAsync(base, 0, sizeof(int64_t) * size_t(M), s));
  COOC_HIP_TRY(hipMemsetAsync(nnz, 0, sizeof(int32_t) * size_t(M), s));
  if (R > 0) k_own_scatter<<<blocks_for(R, 256), 256, 0, s>>>(R, W, part, mbase, mnnz, base, nnz);
  COOC_HIP_TRY(hipGetLastError());
  return Status::Ok();
}

Status launch_merge_owned(hipStream_t s, int32_t M, const int64_t *base, const int32_t *nnz, const int32_t *col,
                          const uint32_t *cnt, const int64_t *rs_all, uint32_t *G, int64_t *grs, int64_t *scal,
                          int64_t observed_window) {
  COOC_HIP_TRY(hipMemsetAsync(scal + 1, 0, sizeof(int64_t), s));
  COOC_HIP_TRY(hipMemsetAsync(scal + 4, 0, sizeof(int64_t), s));
  // the owned rows' entries into the dense global rows (k_merge_global with no row sums: zero deltas); G == NULL: a
  // large universe, whose sparse row slabs the caller merges (launch_gs_merge)
  if (G)
    k_merge_global<<<std::min<unsigned>(blocks_for(int64_t(M) * 64, 256), 8192), 256, 0, s>>>(
        M, base, nnz, col, cnt, nullptr, G, nullptr, nullptr);
  k_add_rowsums<<<std::min<unsigned>(blocks_for(M, 256), 1024), 256, 0, s>>>(M, rs_all, nnz, grs, scal);
  k_finish_scalars<<<1, 1, 0, s>>>(scal, observed_window);
  COOC_HIP_TRY(hipGetLastError());
  return Status::Ok();
}

Status launch_pack_rows(hipStream_t s, int32_t M, const int64_t *base, const int32_t *nnz, const int32_t *col,
                        const uint32_t *cnt, DevBuf &rp, DevBuf &out_col, DevBuf &out_cnt, DevBuf &tmp, int64_t *total) {
  COOC_TRY(rp.reserve(sizeof(int64_t) * (size_t(M) + 1)));
  int64_t *d_rp = rp.as<int64_t>();
  COOC_TRY(tmp.reserve(scan_ws_bytes(M)));
  COOC_HIP_TRY(hipMemsetAsync(d_rp, 0, sizeof(int64_t), s));
  int64_t serr = 0;
  COOC_TRY(launch_scan_ws<true>(ScanI32{nnz}, d_rp + 1, M, tmp.as<unsigned long long>(), &serr, s));
  COOC_HIP_TRY(hipMemcpyAsync(total, d_rp + M, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  if (serr & 8) return Status{2, "internal bounds check failed (row prefix)"};
  COOC_TRY(out_col.reserve(sizeof(int32_t) * size_t(*total + 1)));
  COOC_TRY(out_cnt.reserve(sizeof(uint32_t) * size_t(*total + 1)));
  k_pack_rows<<<std::min<unsigned>(blocks_for(int64_t(M) * 64, 256), 8192), 256, 0, s>>>(
      M, base, nnz, d_rp, col, cnt, out_col.as<int32_t>(), out_cnt.as<uint32_t>());
  COOC_HIP_TRY(hipGetLastError());
  return Status::Ok();
}

Status launch_user_cut(hipStream_t s, int64_t n_users, const int64_t *up, const int32_t *items, int32_t cut,
                       int64_t *cut_ptr, int32_t *cut_items, DevBuf &tmp, int64_t *n_cut) {
  *n_cut = 0;
  if (n_users <= 0) {
    COOC_HIP_TRY(hipMemsetAsync(cut_ptr, 0, sizeof(int64_t), s));
    return Status::Ok();
  }
  // tmp = [capped lengths int64[n_users + 1] | scan workspace] (the scan is not in place)
  const size_t lens_bytes = (sizeof(int64_t) * size_t(n_users + 1) + 255) / 256 * 256;
  COOC_TRY(tmp.reserve(lens_bytes + scan_ws_bytes(n_users)));
  int64_t *lens = tmp.as<int64_t>();
  k_cut_lens<<<blocks_for(n_users, 256), 256, 0, s>>>(n_users, up, cut, lens);
  COOC_HIP_TRY(hipGetLastError());
  COOC_HIP_TRY(hipMemsetAsync(cut_ptr, 0, sizeof(int64_t), s));
  int64_t serr = 0;
  COOC_TRY(launch_scan_ws<true>(ScanI64{lens + 1}, cut_ptr + 1, n_users,
                                reinterpret_cast<unsigned long long *>(static_cast<char *>(tmp.p) + lens_bytes), &serr, s));
  const int64_t waves = std::min<int64_t>(n_users, int64_t(1) << 16);
  k_cut_copy<<<blocks_for(waves * 64, 256), 256, 0, s>>>(n_users, up, items, cut_ptr, cut_items);
  COOC_HIP_TRY(hipGetLastError());
  COOC_HIP_TRY(hipMemcpyAsync(n_cut, cut_ptr + n_users, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  if (serr & 8) return Status{2, "internal bounds check failed (capped list prefix)"};
  return Status::Ok();
}

Status launch_touched(hipStream_t s, int32_t M, const int32_t *row_nnz, int32_t *touched, int64_t *n_touched,
                      DevBuf &tmp) {
  hipcub::CountingInputIterator<int32_t> it(0);
  size_t bytes = 0;
  COOC_HIP_TRY(hipcub::DeviceSelect::If(nullptr, bytes, it, touched, n_touched, M, IsTouched{row_nnz}, s));
  COOC_TRY(tmp.reserve(bytes));
  bytes = tmp.cap;
  COOC_HIP_TRY(hipcub::DeviceSelect::If(tmp.p, bytes, it, touched, n_touched, M, IsTouched{row_nnz}, s));
  return Status::Ok();
}

int rescore_waves_per_block(int32_t topk) { return topk <= 1024 ? 4 : 1; }

size_t rescore_lds_bytes(int32_t topk) {
  const size_t w = size_t(rescore_waves_per_block(topk));
  const size_t heaps = sizeof(double) * (w * size_t(topk + 1) + (w * size_t(topk + 1) + 1) / 2);
  return heaps + w * kRsR * 64 * (sizeof(double) * 2)  // + per-wave score / column / queue rings
         + w * 2 * kRsK * sizeof(double);                 // + the per-wave row tables
}

// k_rescore2: per wave a heap (topk + 1 doubles and ints) and the row's two k11 tables
size_t rescore2_lds_bytes(int32_t topk) {
  const size_t w = 4;
  return sizeof(double) * (w * size_t(topk + 1) + (w * size_t(topk + 1) + 1) / 2) + w * 2 * kRsK * sizeof(double);
}

template <class Rows>
Status launch_rescore_rows(hipStream_t s, const int32_t *rows, const int64_t *n_rows_dev, int64_t max_rows, Rows src,
                           int32_t M, const int64_t *grs, const int64_t *obs, bool exact, int32_t topk,
                           DevBuf &terms, int32_t *out_size, int32_t *out_val, double *out_score) {
  // terms: [ColTerms x M][the rows counter][k11 tables: 2 x 65536 doubles]
  const size_t o_ctr = (sizeof(ColTerms) * size_t(std::max(M, 1)) + 255) & ~size_t(255);
  COOC_TRY(terms.reserve(o_ctr + 256 + sizeof(double) * 2 * 65536));
  auto *row_ctr = reinterpret_cast<unsigned long long *>(static_cast<char *>(terms.p) + o_ctr);
  auto *k11t = reinterpret_cast<double *>(static_cast<char *>(terms.p) + o_ctr + 256);
  COOC_HIP_TRY(hipMemsetAsync(row_ctr, 0, sizeof(unsigned long long), s));
  k_col_terms<<<blocks_for(M, 256), 256, 0, s>>>(M, grs, obs, exact ? 1 : 0, terms.as<ColTerms>());
  k_k11_terms<<<256, 256, 0, s>>>(obs, exact ? 1 : 0, k11t);
  const int waves = rescore_waves_per_block(topk);
  const size_t lds = rescore_lds_bytes(topk);
  // COOC_RS_NO_NAN_EXIT=1: every entry scored even behind a NaN heap root (timing the full work; same output)
  const char *nx = getenv("COOC_RS_NO_NAN_EXIT");
  const int32_t no_nan_exit = (nx && nx[0] == '1') ? 1 : 0;
  const char *rbs = getenv("COOC_RS_BATCH");  // rows per counter grab (A/B knob)
  const int32_t rbatch = rbs ? std::max(1, atoi(rbs)) : 4;
  if (lds > 160 * 1024 - 256) return Status{1, "topk too large for the LDS heaps"};
  int dev = 0, n_cu = 256;
  COOC_HIP_TRY(hipGetDevice(&dev));
  COOC_HIP_TRY(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  // COOC_RS_V: 3 (default; CSR rows) k_rescore3, 2 k_rescore2, 1 k_rescore
  static const int ver = getenv("COOC_RS_V") ? atoi(getenv("COOC_RS_V")) : 3;
  if constexpr (std::is_same<Rows, CsrRows>::value) {
    const size_t lds3 = rescore3_lds_bytes(topk);
    if (ver >= 3 && topk <= 1024 && lds3 <= 64 * 1024) {
      // (COOC_RS_EXP: timing experiments, results invalid -- 1 no heap feed, 2 no scoring)
      static const int exp = getenv("COOC_RS_EXP") ? atoi(getenv("COOC_RS_EXP")) : 0;
      auto kern = k_rescore3;
      int per_cu = 1;
      COOC_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * kR3Waves, lds3));
      const int64_t want3 = (max_rows + kR3Waves - 1) / kR3Waves;
      const unsigned grid3 = unsigned(std::max<int64_t>(1, std::min<int64_t>(want3, int64_t(n_cu) * std::max(1, per_cu))));
      kern<<<grid3, 64 * kR3Waves, lds3, s>>>(rows, n_rows_dev, src, grs, terms.as<ColTerms>(), obs, exact ? 1 : 0,
                                              row_ctr, topk, out_size, out_val, out_score, no_nan_exit, rbatch, exp);
      COOC_HIP_TRY(hipGetLastError());
      return Status::Ok();
    }
  }
  const bool v2 = ver >= 2;
  const size_t lds2 = rescore2_lds_bytes(topk);
  if (v2 && topk <= 1024 && lds2 <= 64 * 1024) {
    // k_rescore2: 4 waves per workgroup, as many workgroups as fit (about 6 waves per SIMD)
    int per_cu = 1;
    COOC_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_rescore2<Rows>, 256, lds2));
    const int64_t want2 = (max_rows + 3) / 4;
    const unsigned grid2 = unsigned(std::max<int64_t>(1, std::min<int64_t>(want2, int64_t(n_cu) * std::max(1, per_cu))));
    k_rescore2<Rows><<<grid2, 256, lds2, s>>>(rows, n_rows_dev, src, grs, terms.as<ColTerms>(), k11t, obs, exact ? 1 : 0,
                                              row_ctr, topk, out_size, out_val, out_score, no_nan_exit, rbatch);
    COOC_HIP_TRY(hipGetLastError());
    return Status::Ok();
  }
  if (lds > 64 * 1024)
    COOC_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(k_rescore<Rows>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
  const int64_t want = (max_rows + waves - 1) / waves;
  const unsigned grid = unsigned(std::max<int64_t>(1, std::min<int64_t>(want, int64_t(n_cu) * 8)));
  k_rescore<Rows><<<grid, 64 * waves, lds, s>>>(rows, n_rows_dev, src, grs, terms.as<ColTerms>(), k11t, obs, exact ? 1 : 0,
                                                 row_ctr, topk, out_size, out_val, out_score, no_nan_exit, rbatch);
  COOC_HIP_TRY(hipGetLastError());
  return Status::Ok();
}

Status launch_rescore(hipStream_t s, const int32_t *touched, const int64_t *scal, int32_t M, const uint32_t *G,
                      const int64_t *grs, bool exact, int32_t topk, int32_t max_rows, DevBuf &terms, int32_t *out_size,
                      int32_t *out_val, double *out_score) {
  // scal: [0] touched rows, [2] rescorer observed, [3] exact observed
  return launch_rescore_rows(s, touched, scal, max_rows, DenseRows{G, M}, M, grs, scal + 2, exact, topk, terms,
                             out_size, out_val, out_score);
}

// The two passes (k_rs_bounds, k_rs_score, k_rs_heap) over the batch's CSR rows in row order (rank_of or id).
// terms: [ColTerms x M][counters][k11 tables][scan state][sbase x M][bp x M (kRsB + 1)][scores x nnz]
Status launch_rescore_two_pass(hipStream_t s, int32_t M, CsrRows src, const int32_t *rank_of, const int64_t *grs,
                               const int64_t *obs, bool exact, int32_t topk, int64_t nnz, DevBuf &terms,
                               int32_t *out_size, int32_t *out_val, double *out_score) {
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t o_ctr = al(sizeof(ColTerms) * size_t(std::max(M, 1)));
  const size_t o_k11 = o_ctr + 256;
  const size_t o_state = o_k11 + sizeof(double) * 2 * 65536;
  const size_t o_sbase = al(o_state + sizeof(unsigned long long) * size_t(scan_state_words(M) + 1));
  const size_t o_bp = al(o_sbase + sizeof(int64_t) * size_t(M));
  const size_t o_trow = al(o_bp + sizeof(int32_t) * size_t(M) * (kRsB + 1));
  const size_t o_tcol = al(o_trow + sizeof(double) * size_t(M) * kRsTK * 2);
  const int64_t n_items_ = (((int64_t(M) + 63) >> 6) * (kRsB / 8)) * 8;
  const size_t o_units = al(o_tcol + sizeof(double) * size_t(M) * kRsTK * 2);
  const size_t o_ubase = al(o_units + sizeof(int32_t) * size_t(n_items_ + 1));
  const size_t o_ustate = al(o_ubase + sizeof(int64_t) * size_t(n_items_ + 1));
  const size_t o_umap = al(o_ustate + sizeof(unsigned long long) * size_t(scan_state_words(n_items_ + 1) + 1));
  const int64_t seg_min = getenv("COOC_RS_SPLIT_SEG") ? std::min<int64_t>(kRsSeg, std::max(64, atoi(getenv("COOC_RS_SPLIT_SEG")))) : kRsSeg;
  const int64_t long_min = getenv("COOC_RS_SPLIT_LONG") ? std::max<int64_t>(1, atoll(getenv("COOC_RS_SPLIT_LONG"))) : kRsLong;
  const int64_t n_seg_max = std::max<int64_t>(nnz, 0) / seg_min + std::max<int64_t>(nnz, 0) / long_min + 1;
  const size_t o_nanrow = al(o_umap + sizeof(int32_t) * size_t(n_items_ + std::max<int64_t>(nnz, 0) / kRsP + 1));
  const size_t o_nseg = al(o_nanrow + sizeof(int32_t) * size_t(M));  // (nanrow, then segdone: zeroed together)
  const size_t o_segdone = al(o_nseg + sizeof(int32_t) * size_t(M + 1));
  const size_t o_segp = al(o_segdone + sizeof(int32_t) * size_t(M));
  const size_t o_ncand = al(o_segp + sizeof(int64_t) * size_t(M + 1));
  const size_t o_cand = al(o_ncand + sizeof(int32_t) * size_t(n_seg_max));
  const size_t o_score = al(o_cand + sizeof(uint16_t) * size_t(n_seg_max) * kRsCand);
  COOC_TRY(terms.reserve(o_score + sizeof(uint32_t) * size_t(std::max<int64_t>(nnz, 1))));
  char *base = static_cast<char *>(terms.p);
  auto *ctr = reinterpret_cast<unsigned long long *>(base + o_ctr);  // [0, 8) pass-1 queues, [8] pass-2 rows
  auto *k11t = reinterpret_cast<double *>(base + o_k11);
  auto *state = reinterpret_cast<unsigned long long *>(base + o_state);
  auto *sbase = reinterpret_cast<int64_t *>(base + o_sbase);
  auto *bp = reinterpret_cast<int32_t *>(base + o_bp);
  auto *score = reinterpret_cast<uint32_t *>(base + o_score);
  auto *trow = reinterpret_cast<double *>(base + o_trow);
  auto *units = reinterpret_cast<int32_t *>(base + o_units);
  auto *ubase = reinterpret_cast<int64_t *>(base + o_ubase);
  auto *ustate = reinterpret_cast<unsigned long long *>(base + o_ustate);
  auto *umap = reinterpret_cast<int32_t *>(base + o_umap);
  auto *tcol = reinterpret_cast<double *>(base + o_tcol);
  auto *nanrow = reinterpret_cast<int32_t *>(base + o_nanrow);
  auto *nseg = reinterpret_cast<int32_t *>(base + o_nseg);
  auto *segdone = reinterpret_cast<int32_t *>(base + o_segdone);
  auto *segp = reinterpret_cast<int64_t *>(base + o_segp);
  auto *ncand = reinterpret_cast<int32_t *>(base + o_ncand);
  auto *cand = reinterpret_cast<uint16_t *>(base + o_cand);
  COOC_HIP_TRY(hipMemsetAsync(ctr, 0, 256, s));
  COOC_HIP_TRY(hipMemsetAsync(nanrow, 0, sizeof(int32_t) * size_t(std::max(M, 1)), s));
  COOC_HIP_TRY(hipMemsetAsync(segdone, 0, sizeof(int32_t) * size_t(std::max(M, 1)), s));
  k_col_terms<<<blocks_for(M, 256), 256, 0, s>>>(M, grs, obs, exact ? 1 : 0, terms.as<ColTerms>());
  k_k11_terms<<<256, 256, 0, s>>>(obs, exact ? 1 : 0, k11t);
  COOC_HIP_TRY(hipGetLastError());
  if (M <= 0) return Status::Ok();
  // sbase = the exclusive prefix of the row lengths (the scan's error word after its state; a timed-out look-back
  // is repaired in-kernel and only flagged)
  COOC_HIP_TRY(hipMemsetAsync(state + scan_state_words(M), 0, sizeof(int64_t), s));
  COOC_TRY(launch_scan<false>(ScanI32{src.row_nnz}, sbase, M, state,
                              reinterpret_cast<int64_t *>(state + scan_state_words(M)), s));
  int dev = 0, n_cu = 256;
  COOC_HIP_TRY(hipGetDevice(&dev));
  COOC_HIP_TRY(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  const int32_t bw = int32_t((int64_t(M) + kRsB - 1) / kRsB);
  k_rs_tables<<<unsigned((int64_t(M) * kRsTK + 255) / 256), 256, 0, s>>>(M, src.row_nnz, grs, obs, exact ? 1 : 0, trow,
                                                                          tcol);
  // the work units (the items' entries summed by k_rs_bounds, a scan of their pieces, k_rs_unit_map): at most
  // n_items + nnz / kRsP of them
  const int64_t n_chunks = (int64_t(M) + 63) >> 6, per_q = n_chunks * (kRsB / 8), n_items = per_q * 8;
  COOC_HIP_TRY(hipMemsetAsync(units, 0, sizeof(int32_t) * size_t(n_items + 1), s));
  k_rs_bounds<<<unsigned(std::min<int64_t>((int64_t(M) + 3) / 4, int64_t(n_cu) * 8)), 256, 0, s>>>(M, src, rank_of, bw, bp,
                                                                                                 per_q, units);
  COOC_HIP_TRY(hipMemsetAsync(ustate + scan_state_words(n_items + 1), 0, sizeof(int64_t), s));
  COOC_TRY(launch_scan<false>(ScanUnits{units}, ubase, n_items + 1, ustate,
                              reinterpret_cast<int64_t *>(ustate + scan_state_words(n_items + 1)), s));
  k_rs_unit_map<<<unsigned((n_items + 255) / 256), 256, 0, s>>>(n_items, units, ubase, umap);
  int per_cu1 = 1;  // (a persistent grid: the work comes from the queues)
  COOC_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu1, k_rs_score, 256, 0));
  k_rs_score<<<unsigned(n_cu) * unsigned(std::max(1, per_cu1)), 256, 0, s>>>(M, src, bp, sbase, grs, terms.as<ColTerms>(), k11t, trow, tcol, obs, exact ? 1 : 0,
                                                 ubase, umap, ctr, score, nanrow,
                                                 getenv("COOC_RS_EXP") ? atoi(getenv("COOC_RS_EXP")) : 0);
  COOC_HIP_TRY(hipGetLastError());
  // the long rows' segments (COOC_RS_SPLIT=0: none) and their prefix
  // (test knobs: COOC_RS_SPLIT_LONG / _SEG / _CAP shrink the thresholds so small logs take the split path)
  const bool split = !(getenv("COOC_RS_SPLIT") && getenv("COOC_RS_SPLIT")[0] == '0');
  const int64_t long_thr = getenv("COOC_RS_SPLIT_LONG") ? std::max<int64_t>(1, atoll(getenv("COOC_RS_SPLIT_LONG"))) : kRsLong;
  const int32_t seg_len = getenv("COOC_RS_SPLIT_SEG") ? std::min(kRsSeg, std::max(64, atoi(getenv("COOC_RS_SPLIT_SEG")))) : kRsSeg;
  const int32_t cand_cap = getenv("COOC_RS_SPLIT_CAP") ? std::min(kRsCand, std::max(1, atoi(getenv("COOC_RS_SPLIT_CAP")))) : kRsCand;
  if (split) {
    k_rs_seg_count<<<unsigned((int64_t(M) + 1 + 255) / 256), 256, 0, s>>>(M, src, nanrow, long_thr, seg_len, nseg);
  } else {
    COOC_HIP_TRY(hipMemsetAsync(nseg, 0, sizeof(int32_t) * size_t(M + 1), s));
  }
  COOC_HIP_TRY(hipMemsetAsync(ustate + scan_state_words(int64_t(M) + 1), 0, sizeof(int64_t), s));
  COOC_TRY(launch_scan<false>(ScanI32{nseg}, segp, int64_t(M) + 1, ustate,
                              reinterpret_cast<int64_t *>(ustate + scan_state_words(int64_t(M) + 1)), s));
  const char *nx = getenv("COOC_RS_NO_NAN_EXIT");
  const int32_t no_nan_exit = (nx && nx[0] == '1') ? 1 : 0;
  const size_t lds = sizeof(double) * kR5Waves * size_t(topk + 1) + sizeof(int32_t) * kR5Waves * size_t(topk + 1);
  int per_cu = 1;
  COOC_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_rs_heap, 64 * kR5Waves, lds));
  const int64_t want = (int64_t(M) + kR5Waves - 1) / kR5Waves;
  const unsigned grid = unsigned(std::max<int64_t>(1, std::min<int64_t>(want, int64_t(n_cu) * std::max(1, per_cu))));
  k_rs_heap<<<grid, 64 * kR5Waves, lds, s>>>(M, src, sbase, score, grs, obs, exact ? 1 : 0, ctr + 8, topk,
                                             out_size, out_val, out_score,
                                             no_nan_exit, getenv("COOC_RS_HEAP_SKIP") ? atoll(getenv("COOC_RS_HEAP_SKIP")) : 0,
                                             segp, cand, ncand, segdone, seg_len, cand_cap);
  COOC_HIP_TRY(hipGetLastError());
  return Status::Ok();
}

Status launch_rescore_batch(hipStream_t s, int32_t M, const int64_t *row_base, const int32_t *row_nnz,
                            const int32_t *col, const uint32_t *cnt, const uint32_t *dense, const int64_t *rowsum,
                            bool exact, int32_t topk, int64_t *obs3, DevBuf &terms, int32_t *out_size,
                            int32_t *out_val, double *out_score, const int32_t *rank_of, bool unordered, int64_t nnz,
                            bool whole_log) {
  COOC_HIP_TRY(hipMemsetAsync(obs3, 0, sizeof(int64_t) * 2, s));
  k_observed<<<std::min<unsigned>(blocks_for(M, 256), 1024), 256, 0, s>>>(rowsum, M, obs3);
  COOC_HIP_TRY(hipGetLastError());
  // obs3: [0] rescorer observed, [1] exact, [2] n_rows (= M)
  if (dense)
    return launch_rescore_rows(s, nullptr, obs3 + 2, M, DenseRows{dense, M}, M, rowsum, obs3, exact, topk, terms,
                               out_size, out_val, out_score);
  // the two passes for whole-log row sums (numeric heaps), k_rescore3 otherwise; COOC_RS_TWO_PASS=1 / 0 forces
  const int tp_env = getenv("COOC_RS_TWO_PASS") ? atoi(getenv("COOC_RS_TWO_PASS")) : -1;  // (read per call: tests)
  const bool two_pass = (tp_env < 0 ? whole_log : tp_env != 0) && !unordered && nnz >= 0 && topk <= 1024;
  if (two_pass)
    return launch_rescore_two_pass(s, M, CsrRows{row_base, row_nnz, col, cnt}, rank_of, rowsum, obs3, exact, topk, nnz,
                                   terms, out_size, out_val, out_score);
  return launch_rescore_rows(s, nullptr, obs3 + 2, M, CsrRows{row_base, row_nnz, col, cnt}, M, rowsum, obs3, exact,
                             topk, terms, out_size, out_val, out_score);
}

Status launch_gs_merge(hipStream_t s, int32_t M, const int64_t *drp, const int32_t *dcol, const uint32_t *dcnt,
                       int64_t nnz, GlobalSparse &g, DevBuf &tmp, int64_t *new_cols) {
  // 1. per delta entry: its old-slab position and whether its column is new; the flags' prefix
  //    (newpre[nnz] = the window's new columns)
  COOC_TRY(g.flag.reserve(sizeof(int32_t) * size_t(std::max<int64_t>(nnz, 1))));
  COOC_TRY(g.opos.reserve(sizeof(int64_t) * size_t(std::max<int64_t>(nnz, 1))));
  COOC_TRY(g.newpre.reserve(sizeof(int64_t) * size_t(nnz + 1)));
  COOC_TRY(g.nbase.reserve(sizeof(int64_t) * size_t(M)));
  COOC_TRY(g.chunk_pre.reserve(sizeof(int64_t) * size_t(M + 1) + sizeof(int32_t) * size_t(M)));
  int32_t *flag = g.flag.as<int32_t>();
  int64_t *newpre = g.newpre.as<int64_t>(), *opos = g.opos.as<int64_t>();
  int64_t *chunk_pre = g.chunk_pre.as<int64_t>();
  int32_t *chunks = reinterpret_cast<int32_t *>(chunk_pre + M + 1);
  COOC_HIP_TRY(hipMemsetAsync(newpre, 0, sizeof(int64_t), s));
  int64_t serr = 0, serr2 = 0;
  if (nnz > 0) {
    k_gs_flags<<<blocks_for(nnz, 256), 256, 0, s>>>(M, nnz, drp, dcol, g.base.as<int64_t>(), g.len.as<int32_t>(),
                                                  g.col.as<int32_t>(), flag, opos);
    COOC_TRY(tmp.reserve(scan_ws_bytes(nnz)));
    COOC_TRY(launch_scan_ws<true>(ScanI32{flag}, newpre + 1, nnz, tmp.as<unsigned long long>(), &serr, s));
  }
  COOC_HIP_TRY(hipMemcpyAsync(new_cols, newpre + nnz, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  if (serr & 8) return Status{2, "internal bounds check failed (new-column prefix)"};
  // 2. room for the moved rows' new slabs (at most live + nnz entries): compact, then grow
  const int64_t need = g.live + nnz;
  if (g.bump + need > g.cap) {
    COOC_TRY(compact_global(s, M, g, tmp, std::max<int64_t>(2 * (g.live + need), int64_t(1) << 12)));
  }
  COOC_TRY(g.bump_dev.reserve(sizeof(uint64_t)));
  COOC_HIP_TRY(hipMemcpyAsync(g.bump_dev.p, &g.bump, sizeof(int64_t), hipMemcpyHostToDevice, s));
  k_gs_alloc<<<blocks_for(M, 256), 256, 0, s>>>(M, drp, newpre, g.len.as<int32_t>(), g.nbase.as<int64_t>(),
                                                g.bump_dev.as<unsigned long long>(), chunks);
  // 3. the moved rows' old entries in kGsChunk pieces, then every delta entry
  COOC_HIP_TRY(hipMemsetAsync(chunk_pre, 0, sizeof(int64_t), s));
  COOC_TRY(tmp.reserve(scan_ws_bytes(M)));
  COOC_TRY(launch_scan_ws<true>(ScanI32{chunks}, chunk_pre + 1, M, tmp.as<unsigned long long>(), &serr2, s));
  // (the chunk total is not read back: a fixed grid strides over chunk_pre[M] chunks)
  k_gs_move_all<<<2048, 256, 0, s>>>(M, chunk_pre, drp, dcol, dcnt, newpre, g.nbase.as<int64_t>(), g.base.as<int64_t>(),
                                    g.len.as<int32_t>(), g.col.as<int32_t>(), g.cnt.as<uint32_t>());
  if (nnz > 0)
    k_gs_insert<<<blocks_for(nnz, 256), 256, 0, s>>>(M, nnz, drp, dcol, dcnt, newpre, flag, opos, g.nbase.as<int64_t>(),
                                                    g.base.as<int64_t>(), g.col.as<int32_t>(), g.cnt.as<uint32_t>());
  k_gs_commit<<<blocks_for(M, 256), 256, 0, s>>>(M, drp, newpre, g.nbase.as<int64_t>(), g.base.as<int64_t>(),
                                                 g.len.as<int32_t>());
  COOC_HIP_TRY(hipGetLastError());
  int64_t bump = 0;
  COOC_HIP_TRY(hipMemcpyAsync(&bump, g.bump_dev.p, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  if (serr2 & 8) return Status{2, "internal bounds check failed (moved-chunk prefix)"};
  g.bump = bump;
  g.live += *new_cols;
  return Status::Ok();
}

Status compact_global(hipStream_t s, int32_t M, GlobalSparse &g, DevBuf &tmp, int64_t new_cap) {
  DevBuf col2, cnt2;
  COOC_TRY(col2.reserve(sizeof(int32_t) * size_t(new_cap)));
  COOC_TRY(cnt2.reserve(sizeof(uint32_t) * size_t(new_cap)));
  COOC_TRY(g.nbase.reserve(sizeof(int64_t) * size_t(M + 1)));
  int64_t *nb = g.nbase.as<int64_t>();
  COOC_HIP_TRY(hipMemsetAsync(nb, 0, sizeof(int64_t), s));
  COOC_TRY(tmp.reserve(scan_ws_bytes(M)));
  int64_t serr = 0;
  COOC_TRY(launch_scan_ws<true>(ScanI32{g.len.as<int32_t>()}, nb + 1, M, tmp.as<unsigned long long>(), &serr, s));
  if (g.col.p)
    k_gs_compact<<<std::min<unsigned>(blocks_for(int64_t(M) * 64, 256), 8192), 256, 0, s>>>(
        M, nb, g.base.as<int64_t>(), g.len.as<int32_t>(), g.col.as<int32_t>(), g.cnt.as<uint32_t>(), col2.as<int32_t>(),
        cnt2.as<uint32_t>());
  COOC_HIP_TRY(hipGetLastError());
  COOC_HIP_TRY(hipStreamSynchronize(s));
  if (serr & 8) {
    col2.release();
    cnt2.release();
    return Status{2, "internal bounds check failed (row slab prefix)"};
  }
  g.col.release();
  g.cnt.release();
  g.col = col2;
  g.cnt = cnt2;
  col2.p = cnt2.p = nullptr;
  col2.cap = cnt2.cap = 0;
  g.cap = new_cap;
  g.bump = g.live;
  return Status::Ok();
}

Status launch_rescore_sparse(hipStream_t s, const int32_t *touched, const int64_t *scal, int32_t M, const GlobalSparse &g,
                             const int64_t *grs, bool exact, int32_t topk, int32_t max_rows, DevBuf &terms,
                             int32_t *out_size, int32_t *out_val, double *out_score) {
  return launch_rescore_rows(s, touched, scal, max_rows,
                             CsrRows{g.base.as<int64_t>(), g.len.as<int32_t>(), g.col.as<int32_t>(), g.cnt.as<uint32_t>()},
                             M, grs, scal + 2, exact, topk, terms, out_size, out_val, out_score);
}

}  // namespace cooc
