// cooc_scan.h — device-wide prefix sums of the large-universe planner, hand-written for gfx950.
//
// One pass over the input (single-pass "decoupled look-back" scan): 256-thread workgroups take tiles of
// 4,096 elements in the order they start (a counter, so every tile a workgroup waits on already runs);
// a tile loads its elements coalesced (striped) into LDS, each thread scans 16 consecutive ones, the
// workgroup scans the thread totals, and wave 0 looks back over the 64 tiles before it at a time for the
// tile's exclusive prefix.  A tile's status is one 64-bit word, (value << 2) | flag (1: the tile's own
// sum, 2: the inclusive prefix through the tile), so value and flag travel together and relaxed
// agent-scope atomics suffice.  Values must stay below 2^62 (the planner's prefixes: pair work < n^2 with
// n < 2^31 contributions).  A look-back that sees no progress for ~2^24 polls stops waiting and sums the
// tile's prefix straight from the input (exact; it sets bit 16 of *err as a diagnostic, not an error), so a lost
// update can neither hang the GPU nor hand a partial prefix to the kernels that index with it.
//
// Replaces the library scans of the planner's timed path (row-order pair-work prefix `epre` over the
// contributions, the packed region prefix over users, the work-item prefix over rows): the keyBy(itemA)
// regrouping of FlinkCooccurrences.java:151-153 and the per-row loop bounds of
// NonSampledUserInteractionCounterOneInputStreamOperator.java:144-151.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "cooc_device.h"

namespace cooc {

constexpr int kScanThreads = 256, kScanPer = 16, kScanTile = kScanThreads * kScanPer;

// LDS position of tile element e (16 consecutive per thread, one 8-B pad word per thread's run: the blocked
// reads of 64 lanes spread over the banks)
__device__ inline int scan_lds_pos(int e) { return e + (e >> 4); }

__device__ inline uint64_t scan_status_load(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void scan_status_store(unsigned long long *p, uint64_t v) {
  __hip_atomic_store(p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// out[i] (i < n) = sum of in(0..i) (kIncl) or of in(0..i-1); state: ceil(n / kScanTile) + 1 zeroed words (the
// last one is the tile counter); err: the caller's error word.
// kBlocked: a thread loads and stores its 16 consecutive elements directly (vectorised, no LDS staging);
// otherwise striped through LDS (one coalesced access per element).
template <bool kIncl, bool kBlocked, class In, class Out>
__global__ __launch_bounds__(kScanThreads) void k_scan_lookback(In in, Out *__restrict__ out, int64_t n,
                                                                unsigned long long *__restrict__ state,
                                                                int64_t n_tiles, int64_t *__restrict__ err) {
  __shared__ int64_t s_v[kBlocked ? 1 : kScanTile + kScanTile / kScanPer];
  __shared__ int64_t s_w[kScanThreads / 64];
  __shared__ int64_t s_tile, s_excl;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) s_tile = int64_t(atomicAdd(&state[n_tiles], 1ull));
  __syncthreads();
  const int64_t tile = s_tile, base = tile * kScanTile;
  // 1.-2. each thread its 16 consecutive elements, inclusive
  int64_t x[kScanPer], run = 0;
  if constexpr (kBlocked) {
    const int64_t b0 = base + int64_t(tid) * kScanPer;
    if (b0 + kScanPer <= n) {
#pragma unroll
      for (int k = 0; k < kScanPer; k++) x[k] = int64_t(in(b0 + k));
    } else {
#pragma unroll
      for (int k = 0; k < kScanPer; k++) x[k] = b0 + k < n ? int64_t(in(b0 + k)) : int64_t(0);
    }
#pragma unroll
    for (int k = 0; k < kScanPer; k++) {
      run += x[k];
      x[k] = run;
    }
  } else {
#pragma unroll
    for (int j = 0; j < kScanPer; j++) {  // striped (coalesced) loads into LDS
      const int e = j * kScanThreads + tid;
      const int64_t i = base + e;
      s_v[scan_lds_pos(e)] = i < n ? int64_t(in(i)) : int64_t(0);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kScanPer; k++) {
      run += s_v[scan_lds_pos(tid * kScanPer + k)];
      x[k] = run;
    }
  }
  // 3. the workgroup's exclusive prefix of the thread totals
  int64_t inc = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) s_w[wave] = inc;
  __syncthreads();
  int64_t pre = inc - run, total = 0;
#pragma unroll
  for (int w = 0; w < kScanThreads / 64; w++) {
    pre += w < wave ? s_w[w] : 0;
    total += s_w[w];
  }
  // 4. the tile's exclusive prefix: wave 0 publishes the tile sum, then looks back 64 tiles at a time
  if (wave == 0) {
    int64_t excl = 0;
    if (tile == 0) {
      if (lane == 0) scan_status_store(&state[0], (uint64_t(total) << 2) | 2ull);
    } else {
      if (lane == 0) scan_status_store(&state[tile], (uint64_t(total) << 2) | 1ull);
      int64_t p = tile - 1;
      uint32_t polls = 0;
      for (;;) {
        const int64_t q = p - lane;
        const uint64_t w = q >= 0 ? scan_status_load(&state[q]) : 2ull;  // before tile 0: an inclusive 0
        const uint32_t f = uint32_t(w & 3ull);
        const uint64_t m2 = __ballot(f == 2u), m0 = __ballot(f == 0u);
        const int first2 = m2 ? __ffsll((unsigned long long)m2) - 1 : 64;  // the closest inclusive prefix
        const uint64_t upto = first2 >= 63 ? ~0ull : ((2ull << first2) - 1ull);
        if (m0 & upto) {  // a tile in between has not published its sum yet
          if (++polls > (1u << 24)) {
            // no progress: the prefix is summed from the input itself (exact, slow, never the common case),
            // so no kernel downstream ever sees a partial prefix, and nothing waits any longer
            int64_t v = 0;
            for (int64_t i = lane; i < base; i += 64) v += int64_t(in(i));
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            excl = v;
            if (lane == 0) atomicOr(reinterpret_cast<unsigned long long *>(err), 16ull);  // (diagnostic only)
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        int64_t v = lane <= first2 ? int64_t(w >> 2) : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        excl += v;
        if (first2 < 64) break;
        p -= 64;
      }
      if (lane == 0) scan_status_store(&state[tile], (uint64_t(excl + total) << 2) | 2ull);
    }
    if (lane == 0) s_excl = excl;
  }
  __syncthreads();
  const int64_t off = s_excl + pre;
  if constexpr (kBlocked) {
    const int64_t b0 = base + int64_t(tid) * kScanPer;
    if (b0 + kScanPer <= n) {
#pragma unroll
      for (int k = 0; k < kScanPer; k++) out[b0 + k] = Out(off + (kIncl ? x[k] : (k ? x[k - 1] : int64_t(0))));
    } else {
#pragma unroll
      for (int k = 0; k < kScanPer; k++)
        if (b0 + k < n) out[b0 + k] = Out(off + (kIncl ? x[k] : (k ? x[k - 1] : int64_t(0))));
    }
    return;
  }
  // 5. back through LDS (blocked), then striped (coalesced) stores
#pragma unroll
  for (int k = 0; k < kScanPer; k++)
    s_v[scan_lds_pos(tid * kScanPer + k)] = off + (kIncl ? x[k] : (k ? x[k - 1] : int64_t(0)));
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kScanPer; j++) {
    const int e = j * kScanThreads + tid;
    const int64_t i = base + e;
    if (i < n) out[i] = Out(s_v[scan_lds_pos(e)]);
  }
}

// Input views of the planner's scans
struct ScanU64 {
  const uint64_t *p;
  __device__ int64_t operator()(int64_t i) const { return int64_t(p[i]); }
};
struct ScanI64 {
  const int64_t *p;
  __device__ int64_t operator()(int64_t i) const { return p[i]; }
};
struct ScanI32 {
  const int32_t *p;
  __device__ int64_t operator()(int64_t i) const { return int64_t(p[i]); }
};

// Workspace words of one scan of n elements (the tile statuses and the counter).
inline int64_t scan_state_words(int64_t n) { return (n + kScanTile - 1) / kScanTile + 1; }

// out[0, n) = the inclusive (kIncl) or exclusive prefix of in; state holds scan_state_words(n) words.
// blocked: 1 vectorised loads (the default), 0 striped through LDS, -1 the COOC_SCAN_BLOCKED knob.
template <bool kIncl, class In, class Out>
Status launch_scan(In in, Out *out, int64_t n, unsigned long long *state, int64_t *err, hipStream_t s,
                   int blocked = -1) {
  if (n <= 0) return Status::Ok();
  const int64_t n_tiles = (n + kScanTile - 1) / kScanTile;
  if (n_tiles > int64_t(INT32_MAX)) return Status{1, "prefix sum over more than 2^31 tiles"};
  COOC_HIP_TRY(hipMemsetAsync(state, 0, sizeof(unsigned long long) * size_t(n_tiles + 1), s));
  static const bool env_blocked = [] {  // (A/B knob: COOC_SCAN_BLOCKED=0 stages the tile through LDS)
    const char *e = getenv("COOC_SCAN_BLOCKED");
    return !(e && e[0] == '0');
  }();
  if (blocked < 0 ? env_blocked : blocked != 0)
    k_scan_lookback<kIncl, true, In, Out><<<unsigned(n_tiles), kScanThreads, 0, s>>>(in, out, n, state, n_tiles, err);
  else
    k_scan_lookback<kIncl, false, In, Out><<<unsigned(n_tiles), kScanThreads, 0, s>>>(in, out, n, state, n_tiles, err);
  COOC_HIP_TRY(hipGetLastError());
  return Status::Ok();
}

// launch_scan with its workspace at ws (scan_state_words(n) + 1 words: the tile statuses, then the error word);
// the error word is copied to *h_err, valid once the stream has drained (callers check bit 8 after their sync).
template <bool kIncl, class In, class Out>
Status launch_scan_ws(In in, Out *out, int64_t n, unsigned long long *ws, int64_t *h_err, hipStream_t s) {
  *h_err = 0;
  if (n <= 0) return Status::Ok();
  int64_t *err = reinterpret_cast<int64_t *>(ws + scan_state_words(n));
  COOC_HIP_TRY(hipMemsetAsync(err, 0, sizeof(int64_t), s));
  COOC_TRY(launch_scan<kIncl>(in, out, n, ws, err, s));
  COOC_HIP_TRY(hipMemcpyAsync(h_err, err, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  return Status::Ok();
}
inline size_t scan_ws_bytes(int64_t n) { return sizeof(unsigned long long) * size_t(scan_state_words(n) + 1); }

}  // namespace cooc
