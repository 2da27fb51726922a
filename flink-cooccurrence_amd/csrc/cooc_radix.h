// cooc_radix.h — stable LSD radix sort of (key, value) pairs and flag compaction for the large-universe planner,
// hand-written for gfx950 (replacing the library sorts and the select on the C3/C5 step).
//
// The planner regroups the interactions by item (the keyBy(itemA) of FlinkCooccurrences.java:151-153: the
// (item, user) contributions sorted by item, users in order within an item), orders the rows by pair work for the
// work queue, and ranks the items by frequency for the column relabel.  All three are stable sorts of 32- or
// 64-bit keys with 32-bit values over a known bit range.
//
// One pass per 8-bit digit, reduce-then-scan:
//   k_rdx_hist     per 4,096-key tile, the digit counts (LDS atomics), stored digit-major (counts[d][tile]);
//   launch_scan    (cooc_scan.h) the exclusive prefix over (digit, tile): where each tile's run of digit d starts;
//   k_rdx_scatter  per tile, each wave ranks its 1,024 keys in input order (the lanes holding one digit found by
//                  one ballot per digit bit; a per-wave LDS counter per digit), the workgroup adds the waves' and
//                  the digits' prefixes, the tile is staged in LDS in digit order and written out in runs.
// Keys of equal digit keep their input order within a tile and across tiles, so every pass is stable and the
// result equals a stable sort by the bit range (descending: by the complemented bits, equal keys still in input
// order, as hipcub's SortPairsDescending).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "cooc_device.h"
#include "cooc_scan.h"

namespace cooc {

constexpr int kRdxThreads = 256, kRdxPer = 16, kRdxTile = kRdxThreads * kRdxPer, kRdxBits = 8;
constexpr int kRdxBuckets = 1 << kRdxBits;

template <class K>
__device__ inline uint32_t rdx_digit(K k, int shift, uint32_t mask, int32_t desc) {
  const K x = desc ? K(~k) : k;
  return uint32_t(x >> shift) & mask;
}

template <class K>
__global__ __launch_bounds__(kRdxThreads) void k_rdx_hist(const K *__restrict__ keys, int64_t n, int shift,
                                                         uint32_t mask, int32_t desc, int64_t n_tiles,
                                                         int32_t *__restrict__ counts) {
  __shared__ int32_t h[kRdxBuckets];
  const int tid = threadIdx.x;
  h[tid] = 0;
  __syncthreads();
  const int64_t base = int64_t(blockIdx.x) * kRdxTile;
#pragma unroll 4
  for (int j = 0; j < kRdxPer; j++) {
    const int64_t i = base + j * kRdxThreads + tid;
    if (i < n) atomicAdd(&h[rdx_digit(keys[i], shift, mask, desc)], 1);
  }
  __syncthreads();
  counts[int64_t(tid) * n_tiles + blockIdx.x] = h[tid];
}

template <class K, class V>
__global__ __launch_bounds__(kRdxThreads) void k_rdx_scatter(const K *__restrict__ kin, const V *__restrict__ vin,
                                                            K *__restrict__ kout, V *__restrict__ vout, int64_t n,
                                                            int shift, int nbits, int32_t desc, int64_t n_tiles,
                                                            const int32_t *__restrict__ offs) {
  __shared__ int32_t cnt[4][kRdxBuckets];  // per wave: keys of each digit ranked so far, then the wave's prefix
  __shared__ int32_t tpre[kRdxBuckets];    // the tile's exclusive prefix over digits
  __shared__ int32_t gb[kRdxBuckets];      // where the tile's run of each digit starts in the output
  __shared__ int32_t wsum[4];
  __shared__ K sk[kRdxTile];
  __shared__ V sv[kRdxTile];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t mask = (1u << nbits) - 1u;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
#pragma unroll
  for (int w = 0; w < 4; w++) cnt[w][tid] = 0;
  __syncthreads();
  const int64_t tile0 = int64_t(blockIdx.x) * kRdxTile;
  const int64_t base = tile0 + wave * (kRdxTile / 4);
  K key[kRdxPer];
  V val[kRdxPer];
  int32_t rk[kRdxPer];
#pragma unroll
  for (int j = 0; j < kRdxPer; j++) {
    const int64_t i = base + j * 64 + lane;
    key[j] = i < n ? kin[i] : K(0);
    val[j] = i < n ? vin[i] : V(0);
  }
#pragma unroll
  for (int j = 0; j < kRdxPer; j++) {  // in input order: (wave, j, lane)
    const bool valid = base + j * 64 + lane < n;
    const uint32_t d = rdx_digit(key[j], shift, mask, desc);
    uint64_t peers = __ballot(valid);
    for (int b = 0; b < nbits; b++) {
      const bool bit = (d >> b) & 1u;
      const uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    const int32_t c = valid ? cnt[wave][d] : 0;
    rk[j] = c + int32_t(__popcll(peers & lt));
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (valid && (peers & lt) == 0ull) cnt[wave][d] = c + int32_t(__popcll(peers));  // the digit's lowest lane
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  {  // thread d: the waves' prefixes of digit d, the tile's total of d, the scan over digits
    const int d = tid;
    const int32_t a0 = cnt[0][d], a1 = cnt[1][d], a2 = cnt[2][d], a3 = cnt[3][d];
    const int32_t tot = a0 + a1 + a2 + a3;
    int32_t incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int32_t before = 0;
    for (int w = 0; w < wave; w++) before += wsum[w];
    tpre[d] = before + incl - tot;
    gb[d] = d <= int(mask) ? offs[int64_t(d) * n_tiles + blockIdx.x] : 0;
    cnt[0][d] = 0;
    cnt[1][d] = a0;
    cnt[2][d] = a0 + a1;
    cnt[3][d] = a0 + a1 + a2;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kRdxPer; j++) {
    if (base + j * 64 + lane < n) {
      const uint32_t d = rdx_digit(key[j], shift, mask, desc);
      const int32_t lp = tpre[d] + cnt[wave][d] + rk[j];
      sk[lp] = key[j];
      sv[lp] = val[j];
    }
  }
  __syncthreads();
  const int32_t n_valid = int32_t(n - tile0 < kRdxTile ? n - tile0 : kRdxTile);
  for (int e = tid; e < n_valid; e += kRdxThreads) {
    const K k = sk[e];
    const uint32_t d = rdx_digit(k, shift, mask, desc);
    const int64_t pos = int64_t(gb[d]) + (e - tpre[d]);
    kout[pos] = k;
    vout[pos] = sv[e];
  }
}

// Scratch of radix_sort_pairs over n pairs: the other half of the ping-pong, the counts, their prefix, the scan.
template <class K, class V>
inline size_t radix_sort_tmp_bytes(int64_t n) {
  const int64_t n_tiles = (n + kRdxTile - 1) / kRdxTile, nc = n_tiles * kRdxBuckets;
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  return al(sizeof(K) * size_t(n)) + al(sizeof(V) * size_t(n)) + 2 * al(sizeof(int32_t) * size_t(nc)) +
         al(sizeof(unsigned long long) * size_t(scan_state_words(nc) + 1));
}

// Stable sort of (kin, vin)[0, n) by key bits [bit0, bit1) into (kout, vout) (distinct from the inputs, which are
// left unchanged); descending: by the complemented bits.  n < 2^31.  tmp: radix_sort_tmp_bytes<K, V>(n) bytes.
template <class K, class V>
Status radix_sort_pairs(const K *kin, const V *vin, K *kout, V *vout, int64_t n, int bit0, int bit1, bool desc,
                        void *tmp, hipStream_t s) {
  if (n <= 0) return Status::Ok();
  if (n >= (int64_t(1) << 31)) return Status{1, "radix sort of 2^31 or more pairs"};
  if (bit1 <= bit0) {
    COOC_HIP_TRY(hipMemcpyAsync(kout, kin, sizeof(K) * size_t(n), hipMemcpyDeviceToDevice, s));
    COOC_HIP_TRY(hipMemcpyAsync(vout, vin, sizeof(V) * size_t(n), hipMemcpyDeviceToDevice, s));
    return Status::Ok();
  }
  const int64_t n_tiles = (n + kRdxTile - 1) / kRdxTile, nc = n_tiles * kRdxBuckets;
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  char *p = static_cast<char *>(tmp);
  K *kalt = reinterpret_cast<K *>(p);
  p += al(sizeof(K) * size_t(n));
  V *valt = reinterpret_cast<V *>(p);
  p += al(sizeof(V) * size_t(n));
  int32_t *counts = reinterpret_cast<int32_t *>(p);
  p += al(sizeof(int32_t) * size_t(nc));
  int32_t *offs = reinterpret_cast<int32_t *>(p);
  p += al(sizeof(int32_t) * size_t(nc));
  unsigned long long *state = reinterpret_cast<unsigned long long *>(p);
  int64_t *err = reinterpret_cast<int64_t *>(state + scan_state_words(nc));
  COOC_HIP_TRY(hipMemsetAsync(err, 0, sizeof(int64_t), s));
  const int passes = (bit1 - bit0 + kRdxBits - 1) / kRdxBits;
  const K *ks = kin;
  const V *vs = vin;
  for (int q = 0; q < passes; q++) {
    const int shift = bit0 + q * kRdxBits, nbits = bit1 - shift < kRdxBits ? bit1 - shift : kRdxBits;
    const bool to_out = ((passes - 1 - q) & 1) == 0;  // the last pass lands in (kout, vout)
    K *kd = to_out ? kout : kalt;
    V *vd = to_out ? vout : valt;
    k_rdx_hist<K><<<unsigned(n_tiles), kRdxThreads, 0, s>>>(ks, n, shift, (1u << nbits) - 1u, desc ? 1 : 0, n_tiles,
                                                            counts);
    COOC_TRY(launch_scan<false>(ScanI32{counts}, offs, nc, state, err, s));
    k_rdx_scatter<K, V><<<unsigned(n_tiles), kRdxThreads, 0, s>>>(ks, vs, kd, vd, n, shift, nbits, desc ? 1 : 0,
                                                                  n_tiles, offs);
    COOC_HIP_TRY(hipGetLastError());
    ks = kd;
    vs = vd;
  }
  return Status::Ok();
}

// out[0, n_sel) = the indices i < n with flag[i] != 0, ascending; *n_sel_dev = their count.  tmp:
// select_tmp_bytes(n) bytes.
struct ScanFlagU8 {
  const uint8_t *p;
  __device__ int64_t operator()(int64_t i) const { return p[i] != 0 ? 1 : 0; }
};
__global__ inline void k_select_scatter(const uint8_t *__restrict__ flag, int64_t n, const int32_t *__restrict__ pos,
                                        int32_t *__restrict__ out, int32_t *__restrict__ n_sel) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (flag[i]) out[pos[i]] = int32_t(i);
  if (i == n - 1) *n_sel = pos[i] + (flag[i] ? 1 : 0);
}
inline size_t select_tmp_bytes(int64_t n) {
  return ((sizeof(int32_t) * size_t(n) + 255) & ~size_t(255)) + sizeof(unsigned long long) * size_t(scan_state_words(n) + 1);
}
inline Status select_flagged(const uint8_t *flag, int64_t n, int32_t *out, int32_t *n_sel_dev, void *tmp, hipStream_t s) {
  if (n <= 0) {
    COOC_HIP_TRY(hipMemsetAsync(n_sel_dev, 0, sizeof(int32_t), s));
    return Status::Ok();
  }
  int32_t *pos = static_cast<int32_t *>(tmp);
  unsigned long long *state =
      reinterpret_cast<unsigned long long *>(static_cast<char *>(tmp) + ((sizeof(int32_t) * size_t(n) + 255) & ~size_t(255)));
  int64_t *err = reinterpret_cast<int64_t *>(state + scan_state_words(n));
  COOC_HIP_TRY(hipMemsetAsync(err, 0, sizeof(int64_t), s));
  COOC_TRY(launch_scan<false>(ScanFlagU8{flag}, pos, n, state, err, s));
  k_select_scatter<<<unsigned((n + 255) / 256), 256, 0, s>>>(flag, n, pos, out, n_sel_dev);
  COOC_HIP_TRY(hipGetLastError());
  return Status::Ok();
}

}  // namespace cooc
