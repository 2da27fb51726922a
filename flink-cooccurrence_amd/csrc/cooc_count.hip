// cooc_count.hip — the hot path: pair expansion + keyed (itemA, itemB) count reduction on gfx950.
//
// Reference semantics restated (see cooc_device.h for the contribution form):
//   NonSampledUserInteractionCounterOneInputStreamOperator.java:113-165   pair emission
//   ItemRowAggregator.java:26-31                                            per-(itemA, window) row reduce
//   RowSumAggregator.java:25-27,54-71                                       per-(item, window) row-sum reduce
//
// Two planners cover every universe: this file's BATCH planner (n_items < 40,320: one dense LDS row per
// chunk, k_acc_batch, for one-window batches, streaming windows and the C2 records exchange) and the
// LARGE-UNIVERSE planner of cooc_sparse.hip (n_items >= 40,320, or any n_items with
// COOC_FLAG_GENERAL_PLANNER: per-row workgroups over LDS hash / dense-tile chunks, k_sp_main).
// HBM model per window: the ordered pairs P stream 4 B partner ids (mostly served by MALL/L2:
// every user list is re-read once per item in it), 12 B per output entry; see DESIGN.md.
#include <cstdio>
#include <hipcub/hipcub.hpp>

#include "cooc_device.h"
#include "cooc_scan.h"

namespace cooc {

namespace {

constexpr int kAccThreads = 1024;
constexpr int kAccWaves = kAccThreads / 64;
constexpr int kBatchLdsBudget = 160 * 1024 - 1536;  // k_acc_batch: its static LDS is under 1.5 KB


__global__ void k_gather_i32(const int32_t *__restrict__ order, const int32_t *__restrict__ src, int32_t n,
                             int32_t *__restrict__ dst) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[order[i]];
}

__global__ void k_split_rows(const int32_t *__restrict__ row_split, const int32_t *__restrict__ split_slot,
                             int32_t M, int32_t *__restrict__ split_row) {
  const int32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a < M && row_split[a]) split_row[split_slot[a]] = a;
}

__global__ void k_totals(const int32_t *__restrict__ ord_cbase, const int32_t *__restrict__ split_slot, int32_t M,
                         PlanTotals *__restrict__ tot, int32_t *__restrict__ queue) {
  tot->n_chunks = ord_cbase[M];
  tot->n_split = split_slot[M];
  queue[0] = 0;
  queue[1] = 0;
}

// Block-wide sum of a uint64 (kAccThreads threads).
__device__ inline uint64_t block_sum_u64(uint64_t v, uint64_t *s_red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) s_red[wave] = v;
  __syncthreads();
  uint64_t t = 0;
  for (int w = 0; w < kAccWaves; w++) t += s_red[w];
  __syncthreads();
  return t;
}

// Two sums with the barriers of one (s_red: 2 kAccWaves).
__device__ inline uint64_t block_sum2_u64(uint64_t v, uint64_t u, uint64_t *s_red, uint64_t *u_sum) {
  for (int o = 32; o > 0; o >>= 1) {
    v += __shfl_xor(v, o, 64);
    u += __shfl_xor(u, o, 64);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    s_red[wave] = v;
    s_red[kAccWaves + wave] = u;
  }
  __syncthreads();
  uint64_t t = 0, w2 = 0;
  for (int w = 0; w < kAccWaves; w++) {
    t += s_red[w];
    w2 += s_red[kAccWaves + w];
  }
  __syncthreads();
  *u_sum = w2;
  return t;
}

// Two-pass compaction: every wave owns a contiguous column range; pass 1 counts its nonzeros,
// one block scan gives each wave its output offset, pass 2 writes (col, cnt) in column order.
// Two barriers per row instead of two per 1024-column tile.
// Output placement of one compacted (row, column tile): either a fixed base (padded rows: the row's
// capacity region plus the entries of earlier tiles) or, with a bump cursor, an exact-size region
// allocated at compaction time (column-tiled runs), recorded per (row, tile) for the final gather.
struct Place {
  int64_t fixed_base;        // used when bump == nullptr
  unsigned long long *bump;  // device cursor of the bump region, or nullptr
  int64_t bump_cap;          // entries in the bump region
  int64_t *slab = nullptr;   // compact_row_ranges4: the workgroup's slab [cur, end) in LDS (one
                             // global atomic per slab instead of one per row), or nullptr
  int64_t slab_size = 0;     // entries taken per slab (>= the row's nnz)
  unsigned long long *err = nullptr;  // bit 2 set when the region is exhausted
};

// kStore: 0 = no stores (experiments), 1 = plain stores, 2 = sc1 stores (written through, the lines
// dropped from the XCD's L2 so that the output does not evict the partner-id working set), 3 = nt.
template <class Src, int kStore = 1>
__device__ inline uint32_t compact_row_ranges(Src *row, int32_t M, int32_t col_off, int32_t *__restrict__ col_out,
                                              uint32_t *__restrict__ cnt_out, Place place, int64_t *base_used,
                                              uint64_t *sum, uint32_t *s_wave, int64_t *s_base) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int32_t per = ((M + kAccWaves - 1) / kAccWaves + 63) & ~63;
  const int32_t lo = min(M, wave * per), hi = min(M, lo + per);
  uint32_t cnt = 0;
  for (int32_t b = lo + lane; b < hi; b += 64) cnt += uint32_t(__popcll(__ballot(row[b] != 0u)));
  // lanes that skipped the last partial iteration still hold the same count (ballot is wave-wide)
  cnt = __shfl(cnt, 0, 64);
  if (lane == 0) s_wave[wave] = cnt;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kAccWaves; w++) {
    const uint32_t x = s_wave[w];
    off += (w < wave) ? x : 0u;
    tot += x;
  }
  if (place.bump) {
    if (tid == 0) {
      int64_t b = tot ? int64_t(atomicAdd(place.bump, (unsigned long long)tot)) : 0;
      if (b + int64_t(tot) > place.bump_cap) b = -1;  // region exhausted: write nothing, the host reports OOM
      *s_base = b;
    }
    __syncthreads();
  }
  const int64_t out_base = place.bump ? *s_base : place.fixed_base;
  *base_used = out_base;
  const bool write = out_base >= 0;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint64_t my_sum = 0;
  for (int32_t b0 = lo; b0 < hi; b0 += 64) {
    const int32_t b = b0 + lane;
    const uint32_t v = b < hi ? row[b] : 0u;
    const uint64_t m = __ballot(v != 0u);
    if (v) {
      if (kStore && write) {
        const int64_t pos = out_base + off + uint32_t(__popcll(m & lt_mask));
        if (kStore == 2) {
          __hip_atomic_store(col_out + pos, col_off + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(cnt_out + pos, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (kStore == 3) {
          __builtin_nontemporal_store(col_off + b, col_out + pos);
          __builtin_nontemporal_store(v, cnt_out + pos);
        } else {
          col_out[pos] = col_off + b;
          cnt_out[pos] = v;
        }
      }
      row[b] = 0;
      my_sum += v;
    }
    off += uint32_t(__popcll(m));
  }
  __syncthreads();
  *sum = my_sum;
  return tot;
}

// compact_row_ranges over a 16-B aligned uint32 LDS row with 16-B LDS reads: every lane holds 4
// consecutive columns, waves own 256-column-aligned ranges, a lane's output slot is the popcount
// prefix of three ballots (its nonzero count in 0..4, bit by bit).  A quarter of the LDS
// instructions and loop trips of the scalar version.  Columns >= M are never read as counters.
template <int kStore = 1>
__device__ inline uint32_t compact_row_ranges4(uint32_t *row, int32_t M, int32_t *__restrict__ col_out,
                                               uint32_t *__restrict__ cnt_out, Place place, int64_t *base_used,
                                               uint64_t *sum, uint32_t *s_wave, int64_t *s_base) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int32_t per = ((M + kAccWaves - 1) / kAccWaves + 255) & ~255;
  const int32_t lo = min(M, wave * per), hi = min(M, lo + per);
  const uint4 *row4 = reinterpret_cast<const uint4 *>(row);
  auto load = [&](int32_t b, uint32_t v[4]) {
    if (b < hi) {
      const uint4 q = row4[b >> 2];
      v[0] = q.x;
      v[1] = b + 1 < hi ? q.y : 0u;
      v[2] = b + 2 < hi ? q.z : 0u;
      v[3] = b + 3 < hi ? q.w : 0u;
    } else {
      v[0] = v[1] = v[2] = v[3] = 0u;
    }
  };
  uint32_t cnt = 0;
  for (int32_t b0 = lo; b0 < hi; b0 += 256) {
    uint32_t v[4];
    load(b0 + 4 * lane, v);
    cnt += (v[0] != 0u) + (v[1] != 0u) + (v[2] != 0u) + (v[3] != 0u);
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if (lane == 0) s_wave[wave] = cnt;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kAccWaves; w++) {
    const uint32_t x = s_wave[w];
    off += (w < wave) ? x : 0u;
    tot += x;
  }
  if (place.bump) {
    if (tid == 0) {
      int64_t b = 0;
      if (place.slab && tot) {
        if (place.slab[0] + int64_t(tot) > place.slab[1]) {  // the rest of the slab is abandoned
          const int64_t take = max(int64_t(tot), place.slab_size);
          place.slab[0] = int64_t(atomicAdd(place.bump, (unsigned long long)take));
          place.slab[1] = place.slab[0] + take;
        }
        b = place.slab[0];
        place.slab[0] += tot;
      } else if (tot) {
        b = int64_t(atomicAdd(place.bump, (unsigned long long)tot));
      }
      if (b + int64_t(tot) > place.bump_cap) {  // region exhausted: write nothing, the host reports OOM
        b = -1;
        if (place.err) atomicOr(place.err, 4ull);
      }
      *s_base = b;
    }
    __syncthreads();
  }
  const int64_t out_base = place.bump ? *s_base : place.fixed_base;
  *base_used = out_base;
  const bool write = out_base >= 0;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint64_t my_sum = 0;
  for (int32_t b0 = lo; b0 < hi; b0 += 256) {
    const int32_t b = b0 + 4 * lane;
    uint32_t v[4];
    load(b, v);
    const uint32_t c = (v[0] != 0u) + (v[1] != 0u) + (v[2] != 0u) + (v[3] != 0u);
    const uint64_t m0 = __ballot(c & 1u), m1 = __ballot(c & 2u), m2 = __ballot(c & 4u);
    const uint32_t pre = uint32_t(__popcll(m0 & lt_mask)) + 2u * uint32_t(__popcll(m1 & lt_mask)) +
                         4u * uint32_t(__popcll(m2 & lt_mask));
    if (c) {
      int64_t pos = out_base + off + pre;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (!v[k]) continue;
        if (kStore && write) {
          if (kStore == 3) {
            __builtin_nontemporal_store(b + k, col_out + pos);
            __builtin_nontemporal_store(v[k], cnt_out + pos);
          } else {
            col_out[pos] = b + k;
            cnt_out[pos] = v[k];
          }
        }
        pos++;
        my_sum += v[k];
      }
      // zero the 4 counters (those >= hi belong to the next wave's range or lie past M: untouched)
      if (b + 3 < hi) {
        reinterpret_cast<uint4 *>(row)[b >> 2] = make_uint4(0u, 0u, 0u, 0u);
      } else {
        for (int k = 0; k < 4 && b + k < hi; k++) row[b + k] = 0u;
      }
    }
    off += uint32_t(__popcll(m0)) + 2u * uint32_t(__popcll(m1)) + 4u * uint32_t(__popcll(m2));
  }
  __syncthreads();
  *sum = my_sum;
  return tot;
}

// ---- 8. split rows: compact the staging rows ------------------------------------------------------
// bump == nullptr: rows go to their padded place row_base[a]; else to an exact-size bump region
// (row_base[a] is set).
__global__ __launch_bounds__(kAccThreads) void k_finalize_split(
    const PlanTotals *__restrict__ tot, const int32_t *__restrict__ split_row, int32_t M,
    uint32_t *__restrict__ staging, int64_t *__restrict__ row_base, int32_t *__restrict__ row_nnz,
    int32_t *__restrict__ col_out, uint32_t *__restrict__ cnt_out, int64_t *__restrict__ split_sum,
    int64_t *__restrict__ err, unsigned long long *__restrict__ bump, int64_t bump_cap) {
  __shared__ uint32_t s_wave[kAccWaves];
  __shared__ uint64_t s_red[kAccWaves];
  __shared__ int64_t s_base;
  const int64_t n_split = tot->n_split;
  for (int64_t s = blockIdx.x; s < n_split; s += gridDim.x) {
    const int32_t a = split_row[s];
    uint64_t sum;
    int64_t used;
    const uint32_t nnz = compact_row_ranges(staging + s * M, M, 0, col_out, cnt_out,
                                            Place{bump ? 0 : row_base[a], bump, bump_cap}, &used, &sum, s_wave,
                                            &s_base);
    const uint64_t total = block_sum_u64(sum, s_red);
    if (threadIdx.x == 0) {
      if (bump) row_base[a] = used;
      row_nnz[a] = int32_t(nnz);
      if (total != uint64_t(split_sum[s])) atomicOr(reinterpret_cast<unsigned long long *>(err), 2ull);
      split_sum[s] = 0;
    }
  }
}

// Sum of row_nnz into tot->nnz_total (which the run zeroed); any grid of 256-thread blocks.
__global__ void k_nnz_total(const int32_t *__restrict__ row_nnz, int32_t M, PlanTotals *__restrict__ tot) {
  __shared__ uint64_t s[4];
  uint64_t v = 0;
  for (int32_t a = blockIdx.x * 256 + threadIdx.x; a < M; a += gridDim.x * 256) v += uint64_t(row_nnz[a]);
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t t = s[0] + s[1] + s[2] + s[3];
    if (t) atomicAdd(reinterpret_cast<unsigned long long *>(&tot->nnz_total), (unsigned long long)t);
  }
}

// Pack: padded CSR -> contiguous CSR (one wave per row).
__global__ void k_pack(const int64_t *__restrict__ row_base, const int64_t *__restrict__ pk_row_ptr,
                       const int32_t *__restrict__ col, const uint32_t *__restrict__ cnt, int32_t M,
                       int32_t *__restrict__ pk_col, uint32_t *__restrict__ pk_cnt) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t a = wave; a < M; a += n_waves) {
    const int64_t src = row_base[a], dst = pk_row_ptr[a], n = pk_row_ptr[a + 1] - dst;
    for (int64_t i = lane; i < n; i += 64) {
      pk_col[dst + i] = col[src + i];
      pk_cnt[dst + i] = cnt[src + i];
    }
  }
}

// ==== batch planner: one window over empty histories, straight from the CSR of user histories =====
// A contribution is (row a, user u) for every interaction (u, a): row a adds u's whole list, then
// -1 at column a (NonSampled...java:129-161 with an empty resident history).  The planner builds
// the row-grouped contribution list as the transpose of A by a counting sort.  Every pass over the
// N interactions is flat (coalesced, balanced whatever the list lengths):
//   k_batch_users    padded lengths pad8(n_u), sum n_u^2, sum n_u pad8(n_u), max n_u
//   k_batch_fill     user index of every interaction (uidx) + the pads of the u16 arena (pad id = M)
//   k_batch_hist     per-block LDS histogram of items over a fixed interaction range + the arena
//   k_batch_colscan  per-item exclusive prefix over the block histograms -> per-block row offsets
//   k_batch_scatter  contribution descriptors (n_u << 40 | arena offset) at their row positions
// and no per-contribution prefix sums: k_acc_batch scans segment lengths inside the workgroup.
constexpr int kPlanThreads = 1024;
constexpr int kPlanUnroll = 4;       // interactions per thread per step of hist / scatter
constexpr int32_t kFillThread = 2048;  // longer lists get a workgroup each in k_batch_fill_long
// Descriptor of a contribution: arena offset (bits 0-39), segment length (bits 40-62), bit 63 set
// for an old position of a streaming window (its segment is the new part; no -1 self term).
constexpr uint64_t kOffMask = (uint64_t(1) << 40) - 1;
constexpr uint64_t kOldPos = uint64_t(1) << 63;
constexpr uint32_t kLenMask = (1u << 23) - 1;

// Per user: padded arena footprint and the contributions' statistics.  old == nullptr: one window
// over empty histories (every position contributes the whole list).  Streaming windows (old[j] =
// resident history length before the window): a user's arena holds the whole list, then (old > 0)
// its new part [old, l) as a second padded segment; new positions contribute the whole list and
// old positions the new part.
__global__ __launch_bounds__(256) void k_batch_users(int64_t U, const int64_t *__restrict__ up,
                                                     const int32_t *__restrict__ old,
                                                     int64_t *__restrict__ plen, PlanTotals *__restrict__ tot) {
  __shared__ uint64_t s2[4], spl[4];
  __shared__ int64_t smax[4];
  const int64_t j = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  uint64_t l2 = 0, lpl = 0;
  int64_t mx = 0;
  if (j < U) {
    const int64_t l = up[j + 1] - up[j];
    const int64_t pl = (l + 7) & ~int64_t(7);
    const int64_t o = old ? int64_t(old[j]) : 0;
    const int64_t pn = o > 0 ? ((l - o + 7) & ~int64_t(7)) : 0;  // padded new part (its own segment)
    plen[j] = pl + pn;
    l2 = uint64_t(l - o) * uint64_t(l) + uint64_t(o) * uint64_t(l - o);
    lpl = uint64_t(l - o) * uint64_t(pl) + uint64_t(o) * uint64_t(pn);
    mx = l;
  }
  for (int o = 32; o > 0; o >>= 1) {
    l2 += __shfl_xor(l2, o, 64);
    lpl += __shfl_xor(lpl, o, 64);
    mx = max(mx, __shfl_xor(mx, o, 64));
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    s2[w] = l2;
    spl[w] = lpl;
    smax[w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 4; k++) {
      l2 += s2[k];
      lpl += spl[k];
      mx = max(mx, smax[k]);
    }
    if (l2) atomicAdd(reinterpret_cast<unsigned long long *>(&tot->sum_l2), (unsigned long long)l2);
    if (lpl) atomicAdd(reinterpret_cast<unsigned long long *>(&tot->sum_lpl), (unsigned long long)lpl);
    if (mx) atomicMax(reinterpret_cast<unsigned long long *>(&tot->max_len), (unsigned long long)mx);
  }
}

// One thread per user: uidx[up[j] .. up[j+1]) = j (16-B stores where aligned) and the arena pads
// [n_j, pad8(n_j)).  Lists longer than kFillThread are queued for k_batch_fill_long.
__global__ __launch_bounds__(256) void k_batch_fill(int64_t U, const int64_t *__restrict__ up,
                                                    const int32_t *__restrict__ old,
                                                    const int64_t *__restrict__ poff, int32_t M,
                                                    int32_t *__restrict__ uidx, uint16_t *__restrict__ arena,
                                                    int32_t *__restrict__ long_list, PlanTotals *__restrict__ tot) {
  const int64_t j = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= U) return;
  const int64_t s = up[j], l = up[j + 1] - s, o = poff[j];
  const int64_t pl = (l + 7) & ~int64_t(7);
  for (int64_t i = l; i < pl; i++) arena[o + i] = uint16_t(M);
  const int64_t h = old ? int64_t(old[j]) : 0;
  if (h > 0)
    for (int64_t i = l - h; i < ((l - h + 7) & ~int64_t(7)); i++) arena[o + pl + i] = uint16_t(M);
  if (l > kFillThread) {
    long_list[atomicAdd(reinterpret_cast<unsigned long long *>(&tot->n_long), 1ull)] = int32_t(j);
    return;
  }
  const int32_t v = int32_t(j);
  int64_t p = s;
  const int64_t e = s + l;
  for (; p < e && (p & 3); p++) uidx[p] = v;
  for (; p + 4 <= e; p += 4) *reinterpret_cast<int4 *>(uidx + p) = make_int4(v, v, v, v);
  for (; p < e; p++) uidx[p] = v;
}

__global__ __launch_bounds__(256) void k_batch_fill_long(const int64_t *__restrict__ up,
                                                         const int32_t *__restrict__ long_list,
                                                         const PlanTotals *__restrict__ tot,
                                                         int32_t *__restrict__ uidx) {
  const int64_t n_long = tot->n_long;
  for (int64_t k = blockIdx.x; k < n_long; k += gridDim.x) {
    const int32_t j = long_list[k];
    const int64_t s = up[j], e = up[j + 1];
    for (int64_t p = s + threadIdx.x; p < e; p += blockDim.x) uidx[p] = j;
  }
}

// Streaming windows: the active users' histories (resident int32 arena, user j at hoff[j]) as
// one CSR over the contribution slots.
__global__ __launch_bounds__(256) void k_window_items(int64_t n, const int64_t *__restrict__ up,
                                                      const int32_t *__restrict__ uidx,
                                                      const int64_t *__restrict__ hoff,
                                                      const int32_t *__restrict__ harena,
                                                      int32_t *__restrict__ items) {
  const int64_t p = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int32_t j = uidx[p];
  items[p] = harena[hoff[j] + (p - up[j])];
}

// Interaction range of partition block b (the same in hist and scatter).
__device__ inline void block_range(int64_t n, int32_t B, int32_t b, int64_t *p0, int64_t *p1) {
  *p0 = n * b / B;
  *p1 = n * (b + 1) / B;
}

__global__ __launch_bounds__(kPlanThreads) void k_batch_hist(int64_t n, int32_t B, const int64_t *__restrict__ up,
                                                             const int32_t *__restrict__ items,
                                                             const int32_t *__restrict__ uidx,
                                                             const int64_t *__restrict__ poff, int32_t M,
                                                             const int32_t *__restrict__ old,
                                                             uint16_t *__restrict__ arena, int32_t *__restrict__ bh,
                                                             PlanTotals *__restrict__ tot) {
  extern __shared__ uint32_t hist[];  // [M]
  const int tid = threadIdx.x, b = blockIdx.x;
  for (int32_t a = tid; a < M; a += kPlanThreads) hist[a] = 0;
  __syncthreads();
  int64_t p0, p1;
  block_range(n, B, b, &p0, &p1);
  bool bad = false;
  for (int64_t pb = p0; pb < p1; pb += int64_t(kPlanThreads) * kPlanUnroll) {
    int32_t it[kPlanUnroll], j[kPlanUnroll];
#pragma unroll
    for (int k = 0; k < kPlanUnroll; k++) {
      const int64_t p = pb + k * kPlanThreads + tid;
      it[k] = p < p1 ? items[p] : -1;
      j[k] = p < p1 ? uidx[p] : -1;
    }
    int64_t dst[kPlanUnroll], dst2[kPlanUnroll];
#pragma unroll
    for (int k = 0; k < kPlanUnroll; k++) {
      const int64_t p = pb + k * kPlanThreads + tid;
      dst[k] = -1;
      dst2[k] = -1;
      if (j[k] >= 0) {
        const int64_t s0 = up[j[k]], i = p - s0;
        dst[k] = poff[j[k]] + i;
        if (old) {  // a new position is also the (i - h)-th id of the user's new-part segment
          const int64_t h = old[j[k]];
          if (h > 0 && i >= h) dst2[k] = dst[k] - i + ((up[j[k] + 1] - s0 + 7) & ~int64_t(7)) + (i - h);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kPlanUnroll; k++) {
      if (dst[k] < 0) continue;
      uint16_t v = uint16_t(M);
      if (uint32_t(it[k]) < uint32_t(M)) {
        atomicAdd(&hist[it[k]], 1u);
        v = uint16_t(it[k]);
      } else {
        bad = true;
      }
      arena[dst[k]] = v;
      if (dst2[k] >= 0) arena[dst2[k]] = v;
    }
  }
  if (bad) atomicOr(reinterpret_cast<unsigned long long *>(&tot->err), 1ull);
  __syncthreads();
  int32_t *row = bh + int64_t(b) * M;
  for (int32_t a = tid; a < M; a += kPlanThreads) row[a] = int32_t(hist[a]);
}

// Column-wise exclusive prefix over the B block histograms (in place); rcnt[a] = column total.
__global__ void k_batch_colscan(int32_t B, int32_t M, int32_t *__restrict__ bh, int32_t *__restrict__ rcnt) {
  const int32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= M) return;
  int32_t run = 0;
  int32_t b = 0;
  for (; b + 8 <= B; b += 8) {
    int32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = bh[int64_t(b + k) * M + a];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      bh[int64_t(b + k) * M + a] = run;
      run += v[k];
    }
  }
  for (; b < B; b++) {
    const int32_t v = bh[int64_t(b) * M + a];
    bh[int64_t(b) * M + a] = run;
    run += v;
  }
  rcnt[a] = run;
}

// ---- owner-major row order of the sharded records path (owner(a) = a mod W) --------------------
// Row a sits at perm_rows(a) = (rows of owners < a mod W) + a / W; W == 1 is the identity.
__host__ __device__ inline int32_t owner_rows_before(int32_t o, int32_t M, int32_t W) {
  const int32_t q = M / W, rem = M % W;
  return o * q + (o < rem ? o : rem);
}

__host__ __device__ inline int32_t perm_rows(int32_t a, int32_t M, int32_t W) {
  return owner_rows_before(a % W, M, W) + a / W;
}

__host__ __device__ inline int32_t inv_perm_rows(int32_t k, int32_t M, int32_t W) {
  const int32_t q = M / W, rem = M % W;
  const int32_t big = rem * (q + 1);  // owners < rem hold q + 1 rows
  const int32_t o = k < big ? k / (q + 1) : rem + (k - big) / q;
  return o + (k - owner_rows_before(o, M, W)) * W;
}

struct PermCount {  // row count of the k-th row in owner-major order (a launch_scan input)
  const int32_t *rcnt;
  int32_t M, W;
  __device__ int64_t operator()(int64_t k) const {
    return int64_t(rcnt[W == 1 ? int32_t(k) : inv_perm_rows(int32_t(k), M, W)]);
  }
};

__global__ void k_perm_counts(const int32_t *__restrict__ rcnt, int32_t M, int32_t W, int32_t *__restrict__ out) {
  const int32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < M) out[k] = rcnt[inv_perm_rows(k, M, W)];
}

// send[o] = descriptors bound for owner o; send[W] = the padded arena size (ids).
__global__ void k_send_counts(const int64_t *__restrict__ row_ptr, const int64_t *__restrict__ arena_ids, int32_t M,
                              int32_t W, int64_t *__restrict__ send) {
  const int32_t o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o < W) send[o] = row_ptr[owner_rows_before(o + 1, M, W)] - row_ptr[owner_rows_before(o, M, W)];
  if (o == 0) send[W] = *arena_ids;
}

// Owner side: contributions of owned row r over all sources.
__global__ void k_sources_sum(const int32_t *__restrict__ recv_counts, int32_t W, int32_t R,
                              int32_t *__restrict__ rcnt) {
  const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  int32_t t = 0;
  for (int32_t s = 0; s < W; s++) t += recv_counts[int64_t(s) * R + r];
  rcnt[r] = t;
}

// Owner side: one workgroup per (source, owned row) segment copies it to its place in the row's
// concatenated list (sources in order), moving each offset into the all-gathered arena (source s at
// s * stride), and accumulates the contributions' statistics for the chunk plan.  A workgroup per
// segment keeps the hot rows' segments (up to ~1e5 records each) from serialising on one wave.
__global__ __launch_bounds__(1024) void k_reorder_sources(const int32_t *__restrict__ recv_counts,
                                                          const int64_t *__restrict__ seg_off,
                                                          const uint64_t *__restrict__ recv_desc,
                                                          const int64_t *__restrict__ row_ptr, int32_t W, int32_t R,
                                                          int64_t stride, uint64_t *__restrict__ desc,
                                                          PlanTotals *__restrict__ tot) {
  __shared__ uint64_t s_red[3][16];
  __shared__ int64_t s_dst;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t K = int64_t(W) * R;
  uint64_t l_sum = 0, lpl_sum = 0, l_max = 0;
  for (int64_t k = blockIdx.x; k < K; k += gridDim.x) {
    const int32_t s = int32_t(k / R), r = int32_t(k % R);
    const int32_t c = recv_counts[k];
    if (c == 0) continue;  // uniform over the workgroup
    if (tid == 0) {
      int64_t dst = row_ptr[r];
      for (int32_t q = 0; q < s; q++) dst += recv_counts[int64_t(q) * R + r];
      s_dst = dst;
    }
    __syncthreads();
    const int64_t dst = s_dst, src = seg_off[k];
    const uint64_t shift = uint64_t(s) * uint64_t(stride);
    for (int32_t i = tid; i < c; i += 1024) {
      const uint64_t d = recv_desc[src + i] + shift;  // offset field: low 40 bits, no carry
      desc[dst + i] = d;
      const uint64_t l = (d >> 40) & kLenMask;
      l_sum += l;
      lpl_sum += (l + 7) & ~uint64_t(7);  // sum over contributions of pad8(n_u) = sum_u n_u pad8(n_u)
      l_max = l > l_max ? l : l_max;
    }
    __syncthreads();  // s_dst is rewritten for the next segment
  }
  for (int o = 32; o > 0; o >>= 1) {
    l_sum += __shfl_xor(l_sum, o, 64);
    lpl_sum += __shfl_xor(lpl_sum, o, 64);
    const uint64_t m = __shfl_xor(l_max, o, 64);
    l_max = m > l_max ? m : l_max;
  }
  if (lane == 0) {
    s_red[0][wave] = l_sum;
    s_red[1][wave] = lpl_sum;
    s_red[2][wave] = l_max;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 16; w++) {
      l_sum += s_red[0][w];
      lpl_sum += s_red[1][w];
      l_max = s_red[2][w] > l_max ? s_red[2][w] : l_max;
    }
    if (l_sum) {
      atomicAdd(reinterpret_cast<unsigned long long *>(&tot->sum_l2), (unsigned long long)l_sum);
      atomicAdd(reinterpret_cast<unsigned long long *>(&tot->sum_lpl), (unsigned long long)lpl_sum);
      atomicMax(reinterpret_cast<unsigned long long *>(&tot->max_len), (unsigned long long)l_max);
    }
  }
}

__global__ __launch_bounds__(kPlanThreads) void k_batch_scatter(int64_t n, int32_t B, const int64_t *__restrict__ up,
                                                                const int32_t *__restrict__ items,
                                                                const int32_t *__restrict__ uidx,
                                                                const int64_t *__restrict__ poff,
                                                                const int64_t *__restrict__ row_ptr, int32_t M,
                                                                int32_t W, const int32_t *__restrict__ bh,
                                                                const int32_t *__restrict__ old,
                                                                uint64_t *__restrict__ desc) {
  extern __shared__ uint32_t next_pos[];  // [M] next free position of each row inside this block's share
  const int tid = threadIdx.x, b = blockIdx.x;
  const int32_t *row = bh + int64_t(b) * M;
  // row_ptr is in owner-major row order (perm_rows; the identity when W == 1)
  for (int32_t a = tid; a < M; a += kPlanThreads)
    next_pos[a] = uint32_t(row_ptr[W == 1 ? a : perm_rows(a, M, W)] + row[a]);
  __syncthreads();
  int64_t p0, p1;
  block_range(n, B, b, &p0, &p1);
  for (int64_t pb = p0; pb < p1; pb += int64_t(kPlanThreads) * kPlanUnroll) {
    int32_t it[kPlanUnroll], j[kPlanUnroll];
#pragma unroll
    for (int k = 0; k < kPlanUnroll; k++) {
      const int64_t p = pb + k * kPlanThreads + tid;
      it[k] = p < p1 ? items[p] : -1;
      j[k] = p < p1 ? uidx[p] : -1;
    }
    uint64_t d[kPlanUnroll];
#pragma unroll
    for (int k = 0; k < kPlanUnroll; k++) {
      d[k] = 0;
      if (j[k] < 0) continue;
      const int64_t s0 = up[j[k]], l = up[j[k] + 1] - s0;
      const int64_t h = old ? int64_t(old[j[k]]) : 0;
      if (pb + k * kPlanThreads + tid - s0 < h)  // old position: the new part, no self term
        d[k] = kOldPos | (uint64_t(l - h) << 40) | uint64_t(poff[j[k]] + ((l + 7) & ~int64_t(7)));
      else
        d[k] = (uint64_t(l) << 40) | uint64_t(poff[j[k]]);
    }
#pragma unroll
    for (int k = 0; k < kPlanUnroll; k++)
      if (uint32_t(it[k]) < uint32_t(M)) desc[atomicAdd(&next_pos[it[k]], 1u)] = d[k];
  }
}

// One launch instead of a memset per small buffer (each fill is a launch on the critical path).
__global__ void k_plan_reset(PlanTotals *__restrict__ tot, int64_t *__restrict__ a0, int64_t *__restrict__ b0) {
  if (threadIdx.x == 0) {
    *tot = PlanTotals{};
    *a0 = 0;
    *b0 = 0;
  }
}

__global__ void k_rows_reset(int32_t R, int64_t *__restrict__ rowsum, int32_t *__restrict__ row_nnz,
                             int64_t *__restrict__ row_base, unsigned long long *__restrict__ bump,
                             int32_t *__restrict__ ord_cbase, int32_t *__restrict__ split_slot) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < R) {
    rowsum[i] = 0;
    row_nnz[i] = 0;
  }
  if (i <= R) row_base[i] = 0;
  if (i == 0) {
    bump[0] = 0;
    bump[1] = 0;
    ord_cbase[0] = 0;
    split_slot[0] = 0;
  }
}

// Chunks of a row: equal shares of its contributions, as many as its estimated pair work needs
// (contributions x mean padded list length per contribution).  Heaviest rows first (sort by count).
__global__ void k_batch_plan(const int32_t *__restrict__ rcnt, int32_t M, const PlanTotals *__restrict__ tot,
                             int64_t n, int64_t chunk_work, uint32_t *__restrict__ key, int32_t *__restrict__ order,
                             int32_t *__restrict__ row_nch, int32_t *__restrict__ row_split) {
  const int32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= M) return;
  const double lbar = n > 0 ? double(tot->sum_lpl) / double(n) : 0.0;
  const int32_t c = rcnt[a];
  int32_t nch = 0;
  if (c > 0) {
    const double w = double(c) * lbar;
    nch = int32_t(min(double(c), max(1.0, ceil(w / double(chunk_work)))));
  }
  key[a] = uint32_t(c);
  order[a] = a;
  row_nch[a] = nch;
  row_split[a] = nch > 1 ? 1 : 0;
}

__global__ void k_batch_chunks(const int32_t *__restrict__ order, const int32_t *__restrict__ ord_nch,
                               const int32_t *__restrict__ ord_cbase, const int64_t *__restrict__ row_ptr,
                               const int32_t *__restrict__ split_slot, int32_t M, Chunk *__restrict__ chunks) {
  const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= M) return;
  const int32_t nch = ord_nch[r];
  if (nch == 0) return;
  const int32_t a = order[r];
  const int64_t c0 = row_ptr[a], cnt = row_ptr[a + 1] - c0;
  const int32_t slot = nch > 1 ? split_slot[a] : -1;
  for (int32_t j = 0; j < nch; j++)
    chunks[ord_cbase[r] + j] = Chunk{a, slot, c0 + cnt * j / nch, c0 + cnt * (j + 1) / nch, 0};
}

__device__ inline uint32_t wave_incl_scan_u32(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// Sparse output of k_acc_batch: a workgroup takes kSlabRows * M entries of the bump region at a time.
constexpr int kSlabRows = 4;

// ★ batch accumulate.  Per chunk (row a, contribution range): up to `db` descriptors per batch;
// their group counts (8 ids per 16-B group) are block-scanned into LDS segment starts; walkers of S
// lanes own equal contiguous group ranges (start segment from a table written by the scan) and
// step S groups at a time, U 16-B loads in flight per lane, the next step's loads issued before this
// step's atomics.  Pad ids (= M) land on the sink counter acc[M], so the inner loop has no
// compares: per partner id one shift/mask and one ds_add_u32.  Latency hiding across chunks: the
// next chunk is dequeued when a chunk starts, and its descriptor and first descriptor batch are
// loaded before this chunk's compaction (chunks are queued heaviest first, so a reservation made at
// the start of a long chunk holds back only lighter ones at the tail).
// Output: DENSE = the counts as a dense row-major uint32 [M x M] matrix in HBM (row a written whole
// from LDS with coalesced stores; split rows add their chunks into the zeroed dense row with
// global atomics); otherwise the column-order sparse compaction into a bump-allocated padded CSR.
template <int U, int S, bool DENSE>
__global__ __launch_bounds__(kAccThreads) void k_acc_batch(
    const Chunk *__restrict__ chunks, PlanTotals *__restrict__ tot, int32_t *__restrict__ queue,
    const uint64_t *__restrict__ desc, const uint16_t *__restrict__ arena, int32_t M, int32_t db, int32_t W,
    int32_t part, int32_t *__restrict__ col_out, uint32_t *__restrict__ cnt_out, unsigned long long *__restrict__ bump,
    int64_t bump_cap, int64_t *__restrict__ row_base, int32_t *__restrict__ row_nnz, uint32_t *__restrict__ staging,
    int64_t *__restrict__ split_sum, int64_t *__restrict__ rowsum, uint32_t *__restrict__ dense) {
  constexpr uint32_t kWalkers = kAccThreads / S;
  extern __shared__ __attribute__((aligned(16))) uint32_t acc[];     // [M + 1]: counters, sink at M
  int64_t *s_seg = reinterpret_cast<int64_t *>(acc + ((M + 2) & ~1));  // [db] arena group - group start
  uint32_t *s_vst = reinterpret_cast<uint32_t *>(s_seg + db);          // [db + 1] group starts
  __shared__ int32_t s_chunk;
  __shared__ uint32_t s_wtot[kAccWaves];
  __shared__ uint32_t s_wave[kAccWaves];
  __shared__ uint64_t s_red[2 * kAccWaves];
  __shared__ int64_t s_base;
  __shared__ int64_t s_slab[2];
  __shared__ int32_t s_qstart[kWalkers];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t n_chunks = tot->n_chunks;
  const uint4 *A = reinterpret_cast<const uint4 *>(arena);
  const uint32_t q = uint32_t(tid) / S, ql = uint32_t(tid) % S;
  for (int32_t b = tid; b <= M; b += kAccThreads) acc[b] = 0;
  if (tid == 0) {
    s_chunk = atomicAdd(queue, 1);
    s_slab[0] = s_slab[1] = 0;
  }
  __syncthreads();
  int32_t ch = s_chunk;
  Chunk c = ch < n_chunks ? chunks[ch] : Chunk{0, -1, 0, 0, 0};
  uint64_t d = (tid < db && c.begin + tid < c.end) ? desc[c.begin + tid] : 0;
  while (ch < n_chunks) {
    int32_t nxt = 0;
    if (tid == 0) nxt = atomicAdd(queue, 1);  // lands while this chunk is walked
    uint64_t my_len = 0, my_self = 0;
    for (int64_t b0 = c.begin; b0 < c.end; b0 += db) {
      const int32_t nb = int32_t(min(int64_t(db), c.end - b0));
      uint32_t ng = 0;
      int64_t gsrc = 0;
      if (tid < nb) {
        const uint32_t l = uint32_t(d >> 40) & kLenMask;
        my_len += l;
        my_self += (d & kOldPos) ? 0u : 1u;
        ng = (l + 7) >> 3;
        gsrc = int64_t(d & kOffMask) >> 3;
      }
      const int64_t b1 = b0 + db;
      d = (tid < db && b1 + tid < c.end) ? desc[b1 + tid] : 0;  // next batch, lands during the walk
      const uint32_t incl = wave_incl_scan_u32(ng);
      if (lane == 63) s_wtot[wave] = incl;
      __syncthreads();
      uint32_t pre = 0, total = 0;
#pragma unroll
      for (int w = 0; w < kAccWaves; w++) {
        const uint32_t x = s_wtot[w];
        pre += (w < wave) ? x : 0u;
        total += x;
      }
      if (tid < nb) {
        const uint32_t ex = pre + incl - ng;
        s_vst[tid] = ex;
        s_seg[tid] = gsrc - int64_t(ex);
        // walkers whose range starts inside this segment: lo_q = floor(total q / kWalkers) in [ex, ex + ng)
        const uint32_t q0 = uint32_t((uint64_t(ex) * kWalkers + total - 1) / total);
        const uint32_t q1 = uint32_t((uint64_t(ex + ng) * kWalkers + total - 1) / total);
        for (uint32_t w = q0; w < q1 && w < kWalkers; w++) s_qstart[w] = tid;
      }
      if (tid == 0) s_vst[nb] = total;
      __syncthreads();
      const uint32_t lo = uint32_t((uint64_t(total) * q) / kWalkers);
      const uint32_t hi = uint32_t((uint64_t(total) * (q + 1)) / kWalkers);
      uint32_t g = lo + ql;
      if (g < hi) {
        int32_t cur = s_qstart[q];
        uint32_t next = s_vst[cur + 1];
        int64_t base = s_seg[cur];
        uint4 v[U];
        bool ok[U];
#pragma unroll
        for (int k = 0; k < U; k++) {
          const uint32_t gk = g + uint32_t(S) * k;
          ok[k] = gk < hi;
          if (ok[k]) {
            while (gk >= next) {
              cur++;
              next = s_vst[cur + 1];
              base = s_seg[cur];
            }
            v[k] = A[base + gk];
          }
        }
        for (; g < hi; g += uint32_t(S) * U) {
          uint4 vn[U];
          bool okn[U];
#pragma unroll
          for (int k = 0; k < U; k++) {
            const uint32_t gk = g + uint32_t(S) * (U + k);
            okn[k] = gk < hi;
            if (okn[k]) {
              while (gk >= next) {
                cur++;
                next = s_vst[cur + 1];
                base = s_seg[cur];
              }
              vn[k] = A[base + gk];
            }
          }
#pragma unroll
          for (int k = 0; k < U; k++) {
            if (ok[k]) {
              const uint32_t w4[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
              for (int h = 0; h < 4; h++) {
                atomicAdd(&acc[w4[h] & 0xFFFFu], 1u);
                atomicAdd(&acc[w4[h] >> 16], 1u);
              }
            }
          }
#pragma unroll
          for (int k = 0; k < U; k++) {
            v[k] = vn[k];
            ok[k] = okn[k];
          }
        }
      }
      __syncthreads();
    }
    if (tid == 0) s_chunk = nxt;
    // every contribution at a new position of the row's item has the -1 self term at its column.
    // Rows are local (output) indices; the row's item is part + row * W (W parts of the sharded path).
    uint64_t self_sum;
    const uint64_t len_sum = block_sum2_u64(my_len, my_self, s_red, &self_sum);  // (publishes s_chunk)
    const int64_t n_c = int64_t(self_sum);
    const int64_t chunk_rowsum = int64_t(len_sum) - n_c;
    const int32_t ch2 = s_chunk;
    const Chunk c2 = ch2 < n_chunks ? chunks[ch2] : Chunk{0, -1, 0, 0, 0};
    const uint64_t d2 = (tid < db && c2.begin + tid < c2.end) ? desc[c2.begin + tid] : 0;
    if (tid == 0) {
      acc[M] = 0;
      acc[part + c.row * W] -= uint32_t(n_c);
      atomicAdd(reinterpret_cast<unsigned long long *>(rowsum + c.row), (unsigned long long)chunk_rowsum);
      if (c.split >= 0)
        atomicAdd(reinterpret_cast<unsigned long long *>(split_sum + c.split), (unsigned long long)chunk_rowsum);
    }
    __syncthreads();
    if (DENSE && c.split < 0) {
      uint32_t *dst = dense + int64_t(c.row) * M;
      uint64_t sum = 0;
      uint32_t nnz = 0;
      if ((M & 3) == 0) {  // 16-B LDS reads and HBM stores (rows 16-B aligned)
        uint4 *a4 = reinterpret_cast<uint4 *>(acc);
        uint4 *d4 = reinterpret_cast<uint4 *>(dst);
        for (int32_t q = tid; q < (M >> 2); q += kAccThreads) {
          const uint4 v = a4[q];
          d4[q] = v;
          a4[q] = make_uint4(0u, 0u, 0u, 0u);
          sum += uint64_t(v.x) + v.y + v.z + v.w;
          nnz += (v.x != 0u) + (v.y != 0u) + (v.z != 0u) + (v.w != 0u);
        }
      } else {
        for (int32_t b = tid; b < M; b += kAccThreads) {
          const uint32_t v = acc[b];
          dst[b] = v;
          acc[b] = 0;
          sum += v;
          nnz += v != 0u;
        }
      }
      // a row sum fits 40 bits (uint32 counts over < 2^8 columns per thread), nnz < 2^16 per thread
      const uint64_t both = block_sum_u64((sum << 24) | uint64_t(nnz), s_red);
      if (tid == 0) {
        row_nnz[c.row] = int32_t(both & 0xFFFFFFu);
        if ((both >> 24) != uint64_t(chunk_rowsum))
          atomicOr(reinterpret_cast<unsigned long long *>(&tot->err), 2ull);
      }
    } else if (DENSE) {
      uint32_t *dst = dense + int64_t(c.row) * M;  // zeroed before the launch; k_dense_split_check closes it
      for (int32_t b = tid; b < M; b += kAccThreads) {
        const uint32_t v = acc[b];
        if (v) {
          atomicAdd(dst + b, v);
          acc[b] = 0;
        }
      }
    } else if (c.split < 0) {
      uint64_t sum;
      int64_t used;
      const Place pl{0, bump, bump_cap, s_slab, int64_t(kSlabRows) * M, reinterpret_cast<unsigned long long *>(&tot->err)};
      const uint32_t nnz = compact_row_ranges4<1>(acc, M, col_out, cnt_out, pl, &used, &sum, s_wave,
                                                                  &s_base);
      const uint64_t total = block_sum_u64(sum, s_red);
      if (tid == 0) {
        row_base[c.row] = used;
        row_nnz[c.row] = int32_t(nnz);
        if (total != uint64_t(chunk_rowsum))
          atomicOr(reinterpret_cast<unsigned long long *>(&tot->err), 2ull);
      }
    } else {
      uint32_t *srow = staging + int64_t(c.split) * M;
      for (int32_t b = tid; b < M; b += kAccThreads) {
        const uint32_t v = acc[b];
        if (v) {
          atomicAdd(srow + b, v);
          acc[b] = 0;
        }
      }
    }
    __syncthreads();
    ch = ch2;
    c = c2;
    d = d2;
  }
}

// Dense output: rows of items without interactions (no chunk) are zero; one wave per row.
__global__ void k_zero_empty_rows(const int32_t *__restrict__ rcnt, int32_t R, int32_t M,
                                  uint32_t *__restrict__ dense) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t a = wave; a < R; a += n_waves) {
    if (rcnt[a] != 0) continue;
    uint32_t *d = dense + a * M;
    for (int32_t b = lane; b < M; b += 64) d[b] = 0;
  }
}

// Dense output: the rows that several chunks add into start at zero.
__global__ void k_zero_rows(const int32_t *__restrict__ rows, const PlanTotals *__restrict__ tot, int32_t M,
                            uint32_t *__restrict__ dense) {
  const int64_t n = tot->n_split;
  for (int64_t s = blockIdx.x; s < n; s += gridDim.x) {
    uint32_t *d = dense + int64_t(rows[s]) * M;
    for (int32_t b = threadIdx.x; b < M; b += blockDim.x) d[b] = 0;
  }
}

// Dense output, split rows: entries and the overflow check (row sum == the chunks' closed form).
__global__ __launch_bounds__(kAccThreads) void k_dense_split_check(const int32_t *__restrict__ split_row,
                                                                   PlanTotals *__restrict__ tot, int32_t M,
                                                                   const uint32_t *__restrict__ dense,
                                                                   int64_t *__restrict__ split_sum,
                                                                   int32_t *__restrict__ row_nnz) {
  __shared__ uint64_t s_red[kAccWaves];
  const int64_t n = tot->n_split;
  for (int64_t s = blockIdx.x; s < n; s += gridDim.x) {
    const int32_t a = split_row[s];
    const uint32_t *d = dense + int64_t(a) * M;
    uint64_t sum = 0;
    uint32_t nnz = 0;
    for (int32_t b = threadIdx.x; b < M; b += kAccThreads) {
      const uint32_t v = d[b];
      sum += v;
      nnz += v != 0u;
    }
    const uint64_t both = block_sum_u64((sum << 24) | uint64_t(nnz), s_red);
    if (threadIdx.x == 0) {
      row_nnz[a] = int32_t(both & 0xFFFFFFu);
      if ((both >> 24) != uint64_t(split_sum[s])) atomicOr(reinterpret_cast<unsigned long long *>(&tot->err), 2ull);
      split_sum[s] = 0;
    }
  }
}

// Dense -> packed CSR (copy-out): one workgroup per row, column order, at pk_row_ptr[a].
__global__ __launch_bounds__(kAccThreads) void k_pack_dense(const uint32_t *__restrict__ dense, int32_t M,
                                                            const int64_t *__restrict__ pk_row_ptr,
                                                            int32_t *__restrict__ pk_col,
                                                            uint32_t *__restrict__ pk_cnt) {
  __shared__ uint32_t s_wave[kAccWaves];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int32_t per = ((M + kAccWaves - 1) / kAccWaves + 63) & ~63;
  const int32_t lo = min(M, wave * per), hi = min(M, lo + per);
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int32_t a = blockIdx.x; a < M; a += gridDim.x) {
    const uint32_t *d = dense + int64_t(a) * M;
    uint32_t cnt = 0;
    for (int32_t b = lo + lane; b < hi; b += 64) cnt += uint32_t(__popcll(__ballot(d[b] != 0u)));
    cnt = __shfl(cnt, 0, 64);
    if (lane == 0) s_wave[wave] = cnt;
    __syncthreads();
    uint32_t off = 0;
    for (int w = 0; w < wave; w++) off += s_wave[w];
    const int64_t base = pk_row_ptr[a];
    for (int32_t b0 = lo; b0 < hi; b0 += 64) {
      const int32_t b = b0 + lane;
      const uint32_t v = b < hi ? d[b] : 0u;
      const uint64_t m = __ballot(v != 0u);
      if (v) {
        const int64_t pos = base + off + uint32_t(__popcll(m & lt_mask));
        pk_col[pos] = b;
        pk_cnt[pos] = v;
      }
      off += uint32_t(__popcll(m));
    }
    __syncthreads();
  }
}

inline unsigned blocks_for(int64_t n, int t) { return unsigned((n + t - 1) / t); }

}  // namespace

Status DevBuf::reserve(size_t bytes) {
  if (bytes <= cap) return Status::Ok();
  release();
  size_t want = bytes + bytes / 4 + 256;
  hipError_t e = hipMalloc(&p, want);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    p = nullptr;
    cap = 0;
    return Status{4, "hipMalloc(" + std::to_string(want) + " B) failed: " + hipGetErrorString(e)};
  }
  cap = want;
  return Status::Ok();
}

void DevBuf::release() {
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
}

Status Counter::init(int32_t n_items) {
  if (n_items <= 0) return Status{1, "n_items must be positive"};
  M_ = n_items;
  COOC_HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&h_tot_), sizeof(PlanTotals), hipHostMallocDefault));
  int dev = 0;
  COOC_HIP_TRY(hipGetDevice(&dev));
  COOC_HIP_TRY(hipDeviceGetAttribute(&n_cu_, hipDeviceAttributeMultiprocessorCount, dev));
  // run_sparse (cooc_sparse.hip) sets its own attributes; the batch planner keeps one LDS row
  if (n_items >= kBatchMaxItems) return Status::Ok();
  for (const void *k : {reinterpret_cast<const void *>(k_acc_batch<4, 16, true>),
                        reinterpret_cast<const void *>(k_acc_batch<4, 8, false>)})
    COOC_HIP_TRY(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kBatchLdsBudget));
  for (const void *k : {reinterpret_cast<const void *>(k_batch_hist), reinterpret_cast<const void *>(k_batch_scatter)})
    COOC_HIP_TRY(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, int(sizeof(uint32_t)) * n_items));
  return Status::Ok();
}

void Counter::release() {
  DevBuf *all[] = {&dense_, &bh_, &uidx_, &long_, &rcnt_, &desc_, &keys_in_, &vals_in_, &keys_out_, &vals_out_,
                   &sort_tmp_, &epre_, &row_ptr_, &row_work_, &row_nch_, &row_cap_, &row_split_, &order_keys_,
                   &order_, &ord_nch_, &ord_cbase_, &row_base_, &split_slot_, &split_row_, &chunks_, &tot_, &queue_,
                   &col_, &cnt_, &staging_, &row_nnz_, &rowsum_, &pk_row_ptr_, &pk_col_, &pk_cnt_,
                   &split_sum_, &tarena_, &bump_, &seg_off_, &plen_, &poff_, &send_, &witems_, &sp_arena_, &sp_arena0_, &sp_defer_, &sr_keys_, &sr_ukeys_, &sr_ucnt_, &sr_aux_, &sp_tb_,
                   &sp_roww_, &sp_pstart_, &sp_pdense_, &sp_est_, &sp_queue_, &sp_ownc_, &sp_ownoff_, &sp_pbase_, &sp_scr_, &sp_scr_mid_, &sp_hz_, &sp_spre_, &scan_state_, &sp_ulen_};
  for (DevBuf *b : all) b->release();
  if (h_tot_) (void)hipHostFree(h_tot_);
  h_tot_ = nullptr;
  for (int i = 0; i < 2; i++) {
    if (aux_[i]) (void)hipStreamDestroy(aux_[i]);
    if (ev_join_[i]) (void)hipEventDestroy(ev_join_[i]);
    aux_[i] = nullptr;
    ev_join_[i] = nullptr;
  }
  if (ev_fork_) (void)hipEventDestroy(ev_fork_);
  ev_fork_ = nullptr;
}

Status Counter::read_totals(PlanTotals *t) {
  COOC_HIP_TRY(hipMemcpy(t, tot_.p, sizeof(PlanTotals), hipMemcpyDeviceToHost));
  return Status::Ok();
}

Status Counter::pack(hipStream_t s, int64_t **row_ptr, int32_t **col, uint32_t **cnt) {
  const int32_t M = M_;
  COOC_TRY(pk_row_ptr_.reserve(sizeof(int64_t) * (M + 1)));
  COOC_HIP_TRY(hipMemcpyAsync(h_tot_, tot_.p, sizeof(PlanTotals), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  const int64_t nnz = h_tot_->nnz_total;
  COOC_TRY(pk_col_.reserve(sizeof(int32_t) * (nnz + 1)));
  COOC_TRY(pk_cnt_.reserve(sizeof(uint32_t) * (nnz + 1)));
  size_t b = 0;
  hipcub::TransformInputIterator<int64_t, WidenI64, const int32_t *> nnz64(row_nnz_.as<int32_t>(), WidenI64{});
  COOC_HIP_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, b, nnz64, pk_row_ptr_.as<int64_t>() + 1, M, s));
  COOC_TRY(sort_tmp_.reserve(b));
  b = sort_tmp_.cap;
  COOC_HIP_TRY(hipMemsetAsync(pk_row_ptr_.p, 0, sizeof(int64_t), s));
  COOC_HIP_TRY(hipcub::DeviceScan::InclusiveSum(sort_tmp_.p, b, nnz64, pk_row_ptr_.as<int64_t>() + 1,
                                                M, s));
  if (dense_mode_) {
    k_pack_dense<<<unsigned(std::max<int32_t>(1, std::min<int32_t>(M, 4 * n_cu_))), kAccThreads, 0, s>>>(
        dense_.as<uint32_t>(), M, pk_row_ptr_.as<int64_t>(), pk_col_.as<int32_t>(), pk_cnt_.as<uint32_t>());
  } else {
    k_pack<<<blocks_for(int64_t(M) * 64, 256) < 8192 ? blocks_for(int64_t(M) * 64, 256) : 8192, 256, 0, s>>>(
        row_base_.as<int64_t>(), pk_row_ptr_.as<int64_t>(), const_cast<int32_t *>(last_col()),
        const_cast<uint32_t *>(last_cnt()), M, pk_col_.as<int32_t>(), pk_cnt_.as<uint32_t>());
  }
  COOC_HIP_TRY(hipGetLastError());
  *row_ptr = pk_row_ptr_.as<int64_t>();
  *col = pk_col_.as<int32_t>();
  *cnt = pk_cnt_.as<uint32_t>();
  return Status::Ok();
}

// ---- batch path, phase 1: local plan (arena, row counts, descriptors in owner-major row order) ----
// W > 1 (sharded records): rows are laid out owner by owner (owner(a) = a mod W, perm_rows), so the
// descriptors bound for one owner are contiguous.  W == 1: natural row order.
// Streaming windows (old != nullptr): up = the active users' contribution prefix (history lengths
// after the window), old = their lengths before it, items = the resident int32 history arena with
// user j at hoff[j].
Status Counter::plan_local(int64_t U, const int64_t *up, const int32_t *items, int64_t n, int32_t W, hipStream_t s,
                           uint64_t *desc, uint16_t *arena, int64_t arena_cap, const int32_t *old,
                           const int64_t *hoff) {
  const int32_t M = M_;
  if (!batch_ok()) return Status{1, "the batch path needs n_items < " + std::to_string(kBatchMaxItems)};
  if (n > int64_t(INT32_MAX)) return Status{1, "more than 2^31 interactions in one window"};
  if (U > int64_t(INT32_MAX)) return Status{1, "more than 2^31 users in one window"};
  if (W < 1 || W > M) return Status{1, "n_parts must be in [1, n_items]"};
  // partition blocks of the hist / scatter passes: one per CU, fewer for tiny inputs
  const int32_t B = int32_t(std::max<int64_t>(1, std::min<int64_t>(n_cu_, n / 4096 + 1)));
  const int64_t U1 = std::max<int64_t>(U, 1);
  if (arena_cap < (old ? 2 * n + 14 * U1 + 16 : n + 7 * U1 + 16))
    return Status{1, "arena buffer smaller than n + 7 n_users + 16 ids"};
  if ((old == nullptr) != (hoff == nullptr)) return Status{1, "old and hoff go together"};
  COOC_TRY(tot_.reserve(sizeof(PlanTotals)));
  COOC_TRY(queue_.reserve(sizeof(int32_t) * 4));
  COOC_TRY(plen_.reserve(sizeof(int64_t) * U1));
  COOC_TRY(poff_.reserve(sizeof(int64_t) * (U1 + 1)));
  COOC_TRY(uidx_.reserve(sizeof(int32_t) * (n + 4)));
  COOC_TRY(long_.reserve(sizeof(int32_t) * U1));
  COOC_TRY(bh_.reserve(sizeof(int32_t) * size_t(B) * M));
  COOC_TRY(rcnt_.reserve(sizeof(int32_t) * M));
  COOC_TRY(row_ptr_.reserve(sizeof(int64_t) * (M + 1)));
  PlanTotals *tot = tot_.as<PlanTotals>();
  int64_t *plen = plen_.as<int64_t>(), *poff = poff_.as<int64_t>(), *row_ptr = row_ptr_.as<int64_t>();
  int32_t *bh = bh_.as<int32_t>(), *rcnt = rcnt_.as<int32_t>(), *uidx = uidx_.as<int32_t>();
  k_plan_reset<<<1, 64, 0, s>>>(tot, poff, row_ptr);
  if (U > 0) {
    k_batch_users<<<blocks_for(U, 256), 256, 0, s>>>(U, up, old, plen, tot);
    COOC_HIP_TRY(hipGetLastError());
  }
  // prefix sums (cooc_scan.h): the users' padded lengths -> poff; row counts in owner-major order -> row_ptr
  // (the identity order when W == 1)
  COOC_TRY(scan_state_.reserve(sizeof(unsigned long long) * size_t(scan_state_words(std::max<int64_t>(U1, M)))));
  unsigned long long *scan_st = scan_state_.as<unsigned long long>();
  if (U > 0) COOC_TRY(launch_scan<true>(ScanI64{plen}, poff + 1, U, scan_st, &tot->err, s));
  // padded arena: every list 16-B aligned and padded to 8 ids with the sink id M; one pad group
  // at the end (never referenced by a segment, keeps the last 16-B load in bounds)
  const size_t lds_m = sizeof(uint32_t) * size_t(M);
  if (U > 0) {
    k_batch_fill<<<blocks_for(U, 256), 256, 0, s>>>(U, up, old, poff, M, uidx, arena, long_.as<int32_t>(), tot);
    k_batch_fill_long<<<256, 256, 0, s>>>(up, long_.as<int32_t>(), tot, uidx);
    if (hoff) {  // the window's histories as one CSR
      COOC_TRY(witems_.reserve(sizeof(int32_t) * (n + 1)));
      if (n > 0) k_window_items<<<blocks_for(n, 256), 256, 0, s>>>(n, up, uidx, hoff, items, witems_.as<int32_t>());
      items = witems_.as<int32_t>();
    }
    k_batch_hist<<<B, kPlanThreads, lds_m, s>>>(n, B, up, items, uidx, poff, M, old, arena, bh, tot);
    k_batch_colscan<<<blocks_for(M, 256), 256, 0, s>>>(B, M, bh, rcnt);
  } else {
    COOC_HIP_TRY(hipMemsetAsync(rcnt, 0, sizeof(int32_t) * M, s));
  }
  COOC_HIP_TRY(hipGetLastError());
  COOC_TRY(launch_scan<true>(PermCount{rcnt, M, W}, row_ptr + 1, M, scan_st, &tot->err, s));
  if (U > 0) {
    k_batch_scatter<<<B, kPlanThreads, lds_m, s>>>(n, B, up, items, uidx, poff, row_ptr, M, W, bh, old, desc);
    COOC_HIP_TRY(hipGetLastError());
  }
  return Status::Ok();
}

// ---- batch path, phase 2: accumulate R rows (row r = global item part + r * W) whose contributions
// are desc[row_ptr[r] .. row_ptr[r + 1]); tot already holds the contributions' statistics
// (sum_l2 = sum of list lengths, sum_lpl, max_len, err).  Synchronises `s` once.
// n = contributions, n_self = those at a new position (each carries the -1 self term); sparse_only
// forces the padded CSR output (streaming windows: the delta rows are merged from it).
Status Counter::accumulate_rows(int32_t R, int32_t W, int32_t part, const int64_t *row_ptr, const int32_t *rcnt,
                                const uint64_t *desc, const uint16_t *arena, int64_t n, int64_t n_self,
                                bool sparse_only, hipStream_t s, CountResult *out, KernelTimer *timer) {
  const int32_t M = M_;
  const int32_t R1 = std::max<int32_t>(R, 1);
  COOC_TRY(order_keys_.reserve(sizeof(uint64_t) * R1));
  COOC_TRY(row_work_.reserve(sizeof(uint64_t) * R1));
  COOC_TRY(order_.reserve(sizeof(int32_t) * R1 * 2));
  COOC_TRY(row_nch_.reserve(sizeof(int32_t) * R1));
  COOC_TRY(row_split_.reserve(sizeof(int32_t) * R1));
  COOC_TRY(ord_nch_.reserve(sizeof(int32_t) * R1));
  COOC_TRY(ord_cbase_.reserve(sizeof(int32_t) * (R1 + 1)));
  COOC_TRY(split_slot_.reserve(sizeof(int32_t) * (R1 + 1)));
  COOC_TRY(split_row_.reserve(sizeof(int32_t) * R1));
  COOC_TRY(row_base_.reserve(sizeof(int64_t) * (R1 + 1)));
  COOC_TRY(row_nnz_.reserve(sizeof(int32_t) * R1));
  COOC_TRY(rowsum_.reserve(sizeof(int64_t) * R1));
  COOC_TRY(bump_.reserve(sizeof(uint64_t) * 2));
  PlanTotals *tot = tot_.as<PlanTotals>();
  k_rows_reset<<<blocks_for(int64_t(R1) + 1, 256), 256, 0, s>>>(R1, rowsum_.as<int64_t>(), row_nnz_.as<int32_t>(),
                                                                row_base_.as<int64_t>(), bump_.as<unsigned long long>(),
                                                                ord_cbase_.as<int32_t>(), split_slot_.as<int32_t>());
  size_t tmp = 0, q = 0;
  COOC_HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, q, row_work_.as<uint32_t>(),
                                                            order_keys_.as<uint32_t>(), order_.as<int32_t>() + R1,
                                                            order_.as<int32_t>(), R1, 0, 32, s));
  tmp = std::max(tmp, q);
  COOC_TRY(sort_tmp_.reserve(tmp));
  COOC_TRY(scan_state_.reserve(sizeof(unsigned long long) * size_t(scan_state_words(R1))));
  unsigned long long *scan_st = scan_state_.as<unsigned long long>();
  // chunk plan: rows by contribution count, heaviest first
  int32_t *order = order_.as<int32_t>();
  if (R > 0) {
    k_batch_plan<<<blocks_for(R, 256), 256, 0, s>>>(rcnt, R, tot, n, chunk_work_, row_work_.as<uint32_t>(), order + R,
                                                    row_nch_.as<int32_t>(), row_split_.as<int32_t>());
    size_t b = sort_tmp_.cap;
    COOC_HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(sort_tmp_.p, b, row_work_.as<uint32_t>(),
                                                              order_keys_.as<uint32_t>(), order + R, order, R, 0, 32,
                                                              s));
    k_gather_i32<<<blocks_for(R, 256), 256, 0, s>>>(order, row_nch_.as<int32_t>(), R, ord_nch_.as<int32_t>());
  }
  if (R > 0) {
    COOC_TRY(launch_scan<true>(ScanI32{ord_nch_.as<int32_t>()}, ord_cbase_.as<int32_t>() + 1, R, scan_st, &tot->err, s));
    COOC_TRY(launch_scan<true>(ScanI32{row_split_.as<int32_t>()}, split_slot_.as<int32_t>() + 1, R, scan_st, &tot->err,
                               s));
    k_split_rows<<<blocks_for(R, 256), 256, 0, s>>>(row_split_.as<int32_t>(), split_slot_.as<int32_t>(), R,
                                                    split_row_.as<int32_t>());
  }
  k_totals<<<1, 1, 0, s>>>(ord_cbase_.as<int32_t>(), split_slot_.as<int32_t>(), R, tot, queue_.as<int32_t>());
  COOC_HIP_TRY(hipGetLastError());
  COOC_HIP_TRY(hipMemcpyAsync(h_tot_, tot, sizeof(PlanTotals), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  if (h_tot_->err & 1) return Status{1, "item id outside [0, n_items)"};
  if (h_tot_->max_len > int64_t(kLenMask)) return Status{1, "a user history longer than 2^23 - 1 items"};
  const int64_t n_chunks = h_tot_->n_chunks, n_split = h_tot_->n_split;
  const int64_t work_total = h_tot_->sum_l2;
  const int64_t pairs = work_total - n_self;
  // Output layout.  Dense uint32 [R x M] when the pairs cover the matrix (P >= R M / 2: dense is then
  // no larger than the sparse (col, cnt) entries it replaces, and written with plain coalesced row
  // stores) and it fits in 40% of free HBM; else the sparse bump-allocated padded CSR, whose entries
  // are at most min(R M, P).
  const int64_t RM = int64_t(R) * M;
  bool dense = !sparse_only && output_pref_ == 2;
  if (!sparse_only && output_pref_ == 0 && 2 * pairs >= RM) {
    size_t free_b = 0, total_b = 0;
    COOC_HIP_TRY(hipMemGetInfo(&free_b, &total_b));
    dense = size_t(RM) * sizeof(uint32_t) <= free_b / 10 * 4 + dense_.cap;
  }
  dense_mode_ = dense;
  last_rows_ = R;
  if (dense) {
    COOC_TRY(dense_.reserve(sizeof(uint32_t) * size_t(std::max<int64_t>(RM, 1))));
  } else {
    // rows are placed in per-workgroup slabs of kSlabRows * M entries; a slab switch abandons less
    // than one row (< M entries, a quarter of a slab) and every workgroup ends inside one slab
    const int64_t bound = std::max<int64_t>(1, std::min<int64_t>(RM, pairs));
    bump_cap_ = bound + bound / 3 + int64_t(n_cu_) * (kSlabRows + 1) * int64_t(M);
    COOC_TRY(col_.reserve(sizeof(int32_t) * (bump_cap_ + 1)));
    COOC_TRY(cnt_.reserve(sizeof(uint32_t) * (bump_cap_ + 1)));
  }
  if (dense && n_chunks == 0 && RM > 0) COOC_HIP_TRY(hipMemsetAsync(dense_.p, 0, sizeof(uint32_t) * size_t(RM), s));
  if (n_chunks > 0) {
    COOC_TRY(chunks_.reserve(sizeof(Chunk) * (n_chunks + 1)));
    COOC_TRY(split_sum_.reserve(sizeof(int64_t) * (n_split + 9)));
    COOC_HIP_TRY(hipMemsetAsync(split_sum_.p, 0, sizeof(int64_t) * (n_split + 9), s));
    if (dense) {
      // rows without contributions stay all-zero; rows of several chunks are zeroed, then added into
      k_zero_empty_rows<<<std::min<unsigned>(blocks_for(R, 4), 4096), 256, 0, s>>>(rcnt, R, M, dense_.as<uint32_t>());
      if (n_split > 0)
        k_zero_rows<<<unsigned(std::min<int64_t>(n_split, 4 * int64_t(n_cu_))), 1024, 0, s>>>(
            split_row_.as<int32_t>(), tot, M, dense_.as<uint32_t>());
      COOC_HIP_TRY(hipGetLastError());
    } else if (n_split > 0) {
      const size_t need = sizeof(uint32_t) * size_t(n_split) * size_t(M);
      COOC_TRY(staging_.reserve(need));
      COOC_HIP_TRY(hipMemsetAsync(staging_.p, 0, need, s));
    }
    k_batch_chunks<<<blocks_for(R, 256), 256, 0, s>>>(order, ord_nch_.as<int32_t>(), ord_cbase_.as<int32_t>(),
                                                      row_ptr, split_slot_.as<int32_t>(), R, chunks_.as<Chunk>());
    COOC_HIP_TRY(hipGetLastError());
    const size_t acc_bytes = sizeof(uint32_t) * size_t((M + 2) & ~1);
    const int db = int(std::min<int64_t>(1024, (int64_t(kBatchLdsBudget) - int64_t(acc_bytes) - 4) / 12));
    if (db < 32) return Status{1, "n_items too large for the LDS row plus descriptors"};
    const size_t lds = acc_bytes + size_t(db) * 12 + 4;
    const int64_t grid = std::min<int64_t>(n_chunks, int64_t(n_cu_));
    // dense rows: 16-lane walkers; sparse rows: 8-lane walkers (profiles/r01: dense/, batch/)
    auto kern = dense_mode_ ? k_acc_batch<4, 16, true> : k_acc_batch<4, 8, false>;
    if (timer && timer->enabled) COOC_HIP_TRY(hipEventRecord(timer->acc_begin, s));
    kern<<<unsigned(grid), kAccThreads, lds, s>>>(chunks_.as<Chunk>(), tot, queue_.as<int32_t>(), desc, arena, M, db,
                                                  W, part, col_.as<int32_t>(), cnt_.as<uint32_t>(),
                                                  bump_.as<unsigned long long>(), bump_cap_, row_base_.as<int64_t>(),
                                                  row_nnz_.as<int32_t>(), staging_.as<uint32_t>(),
                                                  split_sum_.as<int64_t>(), rowsum_.as<int64_t>(),
                                                  dense_.as<uint32_t>());
    COOC_HIP_TRY(hipGetLastError());
    if (timer && timer->enabled) COOC_HIP_TRY(hipEventRecord(timer->acc_end, s));
    if (dense && n_split > 0) {
      k_dense_split_check<<<unsigned(std::min<int64_t>(n_split, 4 * int64_t(n_cu_))), kAccThreads, 0, s>>>(
          split_row_.as<int32_t>(), tot, M, dense_.as<uint32_t>(), split_sum_.as<int64_t>(), row_nnz_.as<int32_t>());
      COOC_HIP_TRY(hipGetLastError());
    } else if (n_split > 0) {
      const int64_t g2 = std::min<int64_t>(n_split, 4 * int64_t(n_cu_));
      k_finalize_split<<<unsigned(g2), kAccThreads, 0, s>>>(
          tot, split_row_.as<int32_t>(), M, staging_.as<uint32_t>(), row_base_.as<int64_t>(),
          row_nnz_.as<int32_t>(), col_.as<int32_t>(), cnt_.as<uint32_t>(), split_sum_.as<int64_t>(),
          reinterpret_cast<int64_t *>(&tot->err), bump_.as<unsigned long long>(), bump_cap_);
      COOC_HIP_TRY(hipGetLastError());
    }
  } else if (timer && timer->enabled) {
    COOC_HIP_TRY(hipEventRecord(timer->acc_begin, s));
    COOC_HIP_TRY(hipEventRecord(timer->acc_end, s));
  }
  if (R > 0) k_nnz_total<<<std::min<unsigned>(blocks_for(R, 256), 64), 256, 0, s>>>(row_nnz_.as<int32_t>(), R, tot);
  COOC_HIP_TRY(hipGetLastError());
  out->row_base = dense ? nullptr : row_base_.as<int64_t>();
  out->row_nnz = row_nnz_.as<int32_t>();
  out->col = dense ? nullptr : col_.as<int32_t>();
  out->cnt = dense ? nullptr : cnt_.as<uint32_t>();
  out->dense = dense ? dense_.as<uint32_t>() : nullptr;
  out->rowsum = rowsum_.as<int64_t>();
  out->work = work_total;
  out->observed = pairs;
  out->nnz = -1;  // known after the stream drains: read_totals().nnz_total
  return Status::Ok();
}

Status Counter::run_batch(int64_t U, const int64_t *up, const int32_t *items, int64_t n, hipStream_t s,
                          CountResult *out, KernelTimer *timer) {
  const int64_t U1 = std::max<int64_t>(U, 1);
  const int64_t arena_cap = n + 7 * U1 + 16;
  COOC_TRY(desc_.reserve(sizeof(uint64_t) * (n + 1)));
  COOC_TRY(tarena_.reserve(sizeof(uint16_t) * arena_cap));
  COOC_TRY(plan_local(U, up, items, n, 1, s, desc_.as<uint64_t>(), tarena_.as<uint16_t>(), arena_cap));
  return accumulate_rows(M_, 1, 0, row_ptr_.as<int64_t>(), rcnt_.as<int32_t>(), desc_.as<uint64_t>(),
                         tarena_.as<uint16_t>(), n, n, false, s, out, timer);
}

// ---- streaming window through the batch planner: the active users' whole histories and new parts
// in a padded u16 arena, one descriptor per history position (new positions: the whole list with
// the self term; old positions: the new part), then the same chunk plan and k_acc_batch.
Status Counter::run_window(const ActiveUsers &au, hipStream_t s, CountResult *out, KernelTimer *timer) {
  const int64_t U = au.n_active, n = au.n_contrib, U1 = std::max<int64_t>(U, 1);
  const int64_t arena_cap = 2 * n + 14 * U1 + 16;
  COOC_TRY(desc_.reserve(sizeof(uint64_t) * (n + 1)));
  COOC_TRY(tarena_.reserve(sizeof(uint16_t) * arena_cap));
  COOC_TRY(plan_local(U, au.cbase, au.arena, n, 1, s, desc_.as<uint64_t>(), tarena_.as<uint16_t>(), arena_cap,
                      au.old, au.off));
  return accumulate_rows(M_, 1, 0, row_ptr_.as<int64_t>(), rcnt_.as<int32_t>(), desc_.as<uint64_t>(),
                         tarena_.as<uint16_t>(), n, au.n_new, true, s, out, timer);
}

// ---- sharded records (W parts): local plan of this part's users -------------------------------
Status Counter::shard_plan(int64_t U, const int64_t *up, const int32_t *items, int64_t n, int32_t W, hipStream_t s,
                           uint64_t *desc, int32_t *row_counts, uint16_t *arena, int64_t arena_cap, int64_t *h_send,
                           int64_t *h_arena_ids, int64_t *h_observed) {
  COOC_TRY(plan_local(U, up, items, n, W, s, desc, arena, arena_cap));
  COOC_TRY(send_.reserve(sizeof(int64_t) * (W + 1)));
  k_perm_counts<<<blocks_for(M_, 256), 256, 0, s>>>(rcnt_.as<int32_t>(), M_, W, row_counts);
  k_send_counts<<<blocks_for(W, 256), 256, 0, s>>>(row_ptr_.as<int64_t>(), poff_.as<int64_t>() + U, M_, W,
                                                   send_.as<int64_t>());
  COOC_HIP_TRY(hipGetLastError());
  std::vector<int64_t> h(W + 1);
  COOC_HIP_TRY(hipMemcpyAsync(h.data(), send_.p, sizeof(int64_t) * (W + 1), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipMemcpyAsync(h_tot_, tot_.p, sizeof(PlanTotals), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  if (h_tot_->err & 1) return Status{1, "item id outside [0, n_items)"};
  for (int32_t o = 0; o < W; o++) h_send[o] = h[o];
  *h_arena_ids = U > 0 ? h[W] : 0;
  *h_observed = h_tot_->sum_l2 - n;
  return Status::Ok();
}

// ---- sharded records: owner side.  recv_counts [W x R] (source-major row counts), recv_desc the
// sources' descriptor segments in source order (offsets into each source's own arena), arena_all
// the all-gathered arenas (source s at s * arena_stride ids).
Status Counter::shard_count(int32_t W, int32_t part, const int32_t *recv_counts, const uint64_t *recv_desc,
                            int64_t n_recv, const uint16_t *arena_all, int64_t arena_stride, hipStream_t s,
                            CountResult *out, KernelTimer *timer) {
  const int32_t M = M_;
  if (!batch_ok()) return Status{1, "the batch path needs n_items < " + std::to_string(kBatchMaxItems)};
  if (W < 1 || part < 0 || part >= W) return Status{1, "part outside [0, n_parts)"};
  if (n_recv > int64_t(INT32_MAX)) return Status{1, "more than 2^31 contributions for one owner"};
  if (arena_stride % 8 != 0) return Status{1, "arena_stride must be a multiple of 8 ids"};
  const int32_t R = M > part ? (M - part + W - 1) / W : 0;
  const int64_t K = int64_t(W) * R;
  COOC_TRY(tot_.reserve(sizeof(PlanTotals)));
  COOC_TRY(queue_.reserve(sizeof(int32_t) * 4));
  COOC_TRY(rcnt_.reserve(sizeof(int32_t) * (R + 1)));
  COOC_TRY(row_ptr_.reserve(sizeof(int64_t) * (R + 1)));
  COOC_TRY(seg_off_.reserve(sizeof(int64_t) * (K + 1)));
  COOC_TRY(desc_.reserve(sizeof(uint64_t) * (n_recv + 1)));
  PlanTotals *tot = tot_.as<PlanTotals>();
  COOC_HIP_TRY(hipMemsetAsync(tot, 0, sizeof(PlanTotals), s));
  COOC_HIP_TRY(hipMemsetAsync(row_ptr_.p, 0, sizeof(int64_t), s));
  if (R > 0) k_sources_sum<<<blocks_for(R, 256), 256, 0, s>>>(recv_counts, W, R, rcnt_.as<int32_t>());
  COOC_HIP_TRY(hipGetLastError());
  hipcub::TransformInputIterator<int64_t, WidenI64, const int32_t *> own64(rcnt_.as<int32_t>(), WidenI64{});
  hipcub::TransformInputIterator<int64_t, WidenI64, const int32_t *> seg64(recv_counts, WidenI64{});
  size_t b1 = 0, b2 = 0;
  COOC_HIP_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, b1, own64, row_ptr_.as<int64_t>() + 1, std::max(R, 1), s));
  COOC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, b2, seg64, seg_off_.as<int64_t>(), int(std::max<int64_t>(K, 1)), s));
  COOC_TRY(sort_tmp_.reserve(std::max(b1, b2)));
  if (R > 0) {
    size_t b = sort_tmp_.cap;
    COOC_HIP_TRY(hipcub::DeviceScan::InclusiveSum(sort_tmp_.p, b, own64, row_ptr_.as<int64_t>() + 1, R, s));
    b = sort_tmp_.cap;
    COOC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(sort_tmp_.p, b, seg64, seg_off_.as<int64_t>(), int(K), s));
    k_reorder_sources<<<unsigned(std::min<int64_t>(K, 8 * int64_t(n_cu_))), 1024, 0, s>>>(
        recv_counts, seg_off_.as<int64_t>(), recv_desc, row_ptr_.as<int64_t>(), W, R, arena_stride,
        desc_.as<uint64_t>(), tot);
    COOC_HIP_TRY(hipGetLastError());
  }
  return accumulate_rows(R, W, part, row_ptr_.as<int64_t>(), rcnt_.as<int32_t>(), desc_.as<uint64_t>(), arena_all,
                         n_recv, n_recv, false, s, out, timer);
}


}  // namespace cooc
