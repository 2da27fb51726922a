// cooc_shard.hip — the owner-partitioned exchange of partial rows (multi-GPU sharding layer).
//
// Users are sharded over GPUs (the reference's keyBy(user), FlinkCooccurrences.java:70); every
// GPU reduces its users' pairs into partial rows (cooc_count.hip).  The reference then re-keys the
// pair records by itemA (keyBy(ItemCooccurrences::getItem), :152) so that one task owns each row;
// here each GPU packs its partial rows by owner(a) = a mod n_parts, the caller moves them with an
// RCCL all-to-all (torch.distributed over xGMI), and the owner merges the n_parts partial rows of
// each of its rows in a dense LDS row (the same accumulator as the hot kernel, weighted adds).
#include <hipcub/hipcub.hpp>

#include "cooc_shard.h"

namespace cooc {
namespace {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;

inline unsigned blocks_for(int64_t n, int t) { return unsigned((n + t - 1) / t); }

// rows owned by part p: a = p, p + n, p + 2n, ... < M
__host__ __device__ inline int32_t rows_owned(int32_t M, int32_t n, int32_t p) {
  return p < M ? (M - p + n - 1) / n : 0;
}

// Row a's position in (owner, row) order.
__device__ inline int32_t perm_index(int32_t a, int32_t M, int32_t n) {
  const int32_t o = a % n, r = a / n;
  // rows of owners < o: every owner o' < o owns rows_owned(M, n, o') rows
  const int32_t q = M / n, rem = M % n;  // owners < rem own q + 1 rows, the rest q
  const int32_t before = o * q + min(o, rem);
  return before + r;
}

__global__ void k_permute_nnz(const int32_t *__restrict__ row_nnz, int32_t M, int32_t n,
                              int32_t *__restrict__ perm_nnz, int64_t *__restrict__ part_entries) {
  const int32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= M) return;
  const int32_t v = row_nnz[a];
  perm_nnz[perm_index(a, M, n)] = v;
  if (v) atomicAdd(reinterpret_cast<unsigned long long *>(part_entries + (a % n)), (unsigned long long)v);
}

// One wave per row: (col, cnt) of the padded CSR -> packed uint64 (col << 32 | cnt) in owner order.
__global__ void k_pack_entries(const int64_t *__restrict__ row_base, const int32_t *__restrict__ row_nnz,
                               const int32_t *__restrict__ col, const uint32_t *__restrict__ cnt,
                               const int64_t *__restrict__ perm_off, int32_t M, int32_t n,
                               uint64_t *__restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t a = wave; a < M; a += n_waves) {
    const int32_t k = row_nnz[a];
    if (!k) continue;
    const int64_t src = row_base[a], dst = perm_off[perm_index(int32_t(a), M, n)];
    for (int32_t i = lane; i < k; i += 64)
      out[dst + i] = (uint64_t(uint32_t(col[src + i])) << 32) | uint64_t(cnt[src + i]);
  }
}

// Dense result: one workgroup per row compacts the row's nonzeros (column order) into the packed
// (col << 32 | cnt) entries of its owner segment.
__global__ __launch_bounds__(kThreads) void k_pack_entries_dense(const uint32_t *__restrict__ dense,
                                                                const int64_t *__restrict__ perm_off, int32_t M,
                                                                int32_t n, uint64_t *__restrict__ out) {
  __shared__ uint32_t s_wave[kWaves];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int32_t per = ((M + kWaves - 1) / kWaves + 63) & ~63;
  const int32_t lo = min(M, wave * per), hi = min(M, lo + per);
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int32_t a = blockIdx.x; a < M; a += gridDim.x) {
    const uint32_t *d = dense + int64_t(a) * M;
    uint32_t c = 0;
    for (int32_t b = lo + lane; b < hi; b += 64) c += uint32_t(__popcll(__ballot(d[b] != 0u)));
    c = __shfl(c, 0, 64);
    if (lane == 0) s_wave[wave] = c;
    __syncthreads();
    uint32_t off = 0;
    for (int w = 0; w < wave; w++) off += s_wave[w];
    const int64_t base = perm_off[perm_index(a, M, n)];
    for (int32_t b0 = lo; b0 < hi; b0 += 64) {
      const int32_t b = b0 + lane;
      const uint32_t v = b < hi ? d[b] : 0u;
      const uint64_t m = __ballot(v != 0u);
      if (v) out[base + off + uint32_t(__popcll(m & lt))] = (uint64_t(uint32_t(b)) << 32) | uint64_t(v);
      off += uint32_t(__popcll(m));
    }
    __syncthreads();
  }
}

// Per owned row r: total received entries (sum over sources) -> output capacity.
__global__ void k_merge_plan(const int32_t *__restrict__ recv_nnz, int32_t n_src, int32_t R, int32_t M,
                             int64_t *__restrict__ cap) {
  const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  int64_t t = 0;
  for (int32_t s = 0; s < n_src; s++) t += recv_nnz[int64_t(s) * R + r];
  cap[r] = t < M ? t : M;
}

// Dense LDS row per owned row; weighted adds of every source's partial row; column-order compaction.
__global__ __launch_bounds__(kThreads) void k_merge_rows(
    const int32_t *__restrict__ recv_nnz, const int64_t *__restrict__ recv_off, const uint64_t *__restrict__ entries,
    int32_t n_src, int32_t R, int32_t M, int32_t part, int32_t n_parts, const int64_t *__restrict__ row_base,
    int32_t *__restrict__ row_nnz, int32_t *__restrict__ col_out, uint32_t *__restrict__ cnt_out,
    const int64_t *__restrict__ rowsum_global, int64_t *__restrict__ rowsum_out, int64_t *__restrict__ err) {
  extern __shared__ uint32_t acc[];
  __shared__ uint32_t s_wave[kWaves];
  __shared__ uint64_t s_red[kWaves];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int32_t b = tid; b < M; b += kThreads) acc[b] = 0;
  __syncthreads();
  for (int32_t r = blockIdx.x; r < R; r += gridDim.x) {
    for (int32_t s = 0; s < n_src; s++) {
      const int64_t k = int64_t(s) * R + r;
      const int64_t lo = recv_off[k], hi = lo + recv_nnz[k];
      for (int64_t i = lo + tid; i < hi; i += kThreads) {
        const uint64_t e = entries[i];
        atomicAdd(&acc[uint32_t(e >> 32)], uint32_t(e));
      }
    }
    __syncthreads();
    // two-pass compaction (as in the hot kernel)
    const int32_t per = ((M + kWaves - 1) / kWaves + 63) & ~63;
    const int32_t lo = min(M, wave * per), hi = min(M, lo + per);
    uint32_t c = 0;
    for (int32_t b = lo + lane; b < hi; b += 64) c += uint32_t(__popcll(__ballot(acc[b] != 0u)));
    c = __shfl(c, 0, 64);
    if (lane == 0) s_wave[wave] = c;
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (int w = 0; w < kWaves; w++) {
      const uint32_t x = s_wave[w];
      off += (w < wave) ? x : 0u;
      tot += x;
    }
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int64_t base = row_base[r];
    uint64_t sum = 0;
    for (int32_t b0 = lo; b0 < hi; b0 += 64) {
      const int32_t b = b0 + lane;
      const uint32_t v = b < hi ? acc[b] : 0u;
      const uint64_t m = __ballot(v != 0u);
      if (v) {
        const int64_t pos = base + off + uint32_t(__popcll(m & lt));
        col_out[pos] = b;
        cnt_out[pos] = v;
        acc[b] = 0;
        sum += v;
      }
      off += uint32_t(__popcll(m));
    }
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if (lane == 0) s_red[wave] = sum;
    __syncthreads();
    if (tid == 0) {
      uint64_t t = 0;
      for (int w = 0; w < kWaves; w++) t += s_red[w];
      row_nnz[r] = int32_t(tot);
      rowsum_out[r] = int64_t(t);
      if (rowsum_global && int64_t(t) != rowsum_global[part + int64_t(r) * n_parts])
        atomicOr(reinterpret_cast<unsigned long long *>(err), 2ull);
    }
    __syncthreads();
  }
}

// ---- large universes (n_items >= kMergeDenseMax: no dense LDS row) --------------------------------------
// Every received entry as the sort key (owned row index << 32 | column) and its count: a segment k = (source,
// owned row r) of the source-major buffers holds one source's partial row r, in column order.
__global__ void k_merge_keys(const int32_t *__restrict__ recv_nnz, const int64_t *__restrict__ recv_off,
                             const uint64_t *__restrict__ entries, int64_t K, int32_t R, uint64_t *__restrict__ keys,
                             uint32_t *__restrict__ vals) {
  const int lane = threadIdx.x & 63;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t k = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; k < K; k += n_waves) {
    const uint64_t r = uint64_t(k % R);
    const int64_t lo = recv_off[k], hi = lo + recv_nnz[k];
    for (int64_t i = lo + lane; i < hi; i += 64) {
      const uint64_t e = entries[i];
      keys[i] = (r << 32) | (e >> 32);
      vals[i] = uint32_t(e);
    }
  }
}

// Owned row r's entries among the merged (sorted, reduced) keys: [lower_bound(r << 32), lower_bound((r+1) << 32)).
__global__ void k_merge_rows_from_keys(const uint64_t *__restrict__ ukeys, const uint32_t *__restrict__ usum,
                                       const int64_t *__restrict__ n_runs_p, int32_t R, int32_t part, int32_t n_parts,
                                       int64_t *__restrict__ row_base, int32_t *__restrict__ row_nnz,
                                       int32_t *__restrict__ col_out, uint32_t *__restrict__ cnt_out,
                                       const int64_t *__restrict__ rowsum_global, int64_t *__restrict__ rowsum_out,
                                       int64_t *__restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  const int64_t n = n_runs_p[0];
  auto lb = [&](uint64_t key) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (ukeys[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
  };
  for (int64_t r = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; r < R; r += n_waves) {
    const int64_t b = lb(uint64_t(r) << 32), e = lb(uint64_t(r + 1) << 32);
    uint64_t sum = 0;
    for (int64_t i = b + lane; i < e; i += 64) {
      col_out[i] = int32_t(uint32_t(ukeys[i]));
      cnt_out[i] = usum[i];
      sum += usum[i];
    }
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if (lane == 0) {
      row_base[r] = b;
      row_nnz[r] = int32_t(e - b);
      rowsum_out[r] = int64_t(sum);
      if (rowsum_global && int64_t(sum) != rowsum_global[part + r * n_parts])
        atomicOr(reinterpret_cast<unsigned long long *>(err), 2ull);
    }
  }
}

}  // namespace

Status Sharder::plan(const CountResult &r, int32_t M, int32_t n_parts, hipStream_t s, int64_t *h_entries) {
  if (n_parts < 1) return Status{1, "n_parts must be >= 1"};
  COOC_TRY(perm_nnz_.reserve(sizeof(int32_t) * (M + 1)));
  COOC_TRY(perm_off_.reserve(sizeof(int64_t) * (M + 1)));
  COOC_TRY(part_entries_.reserve(sizeof(int64_t) * n_parts));
  COOC_HIP_TRY(hipMemsetAsync(part_entries_.p, 0, sizeof(int64_t) * n_parts, s));
  k_permute_nnz<<<blocks_for(M, 256), 256, 0, s>>>(r.row_nnz, M, n_parts, perm_nnz_.as<int32_t>(),
                                                   part_entries_.as<int64_t>());
  COOC_HIP_TRY(hipGetLastError());
  size_t b = 0;
  hipcub::TransformInputIterator<int64_t, WidenI64, const int32_t *> nnz64(perm_nnz_.as<int32_t>(), WidenI64{});
  COOC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, b, nnz64, perm_off_.as<int64_t>(), M, s));
  COOC_TRY(tmp_.reserve(b));
  b = tmp_.cap;
  COOC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp_.p, b, nnz64, perm_off_.as<int64_t>(), M, s));
  COOC_HIP_TRY(hipMemcpyAsync(h_entries, part_entries_.p, sizeof(int64_t) * n_parts, hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  planned_parts_ = n_parts;
  return Status::Ok();
}

Status Sharder::pack(const CountResult &r, int32_t M, int32_t n_parts, hipStream_t s, int32_t *d_row_nnz,
                     uint64_t *d_entries) {
  if (n_parts != planned_parts_) return Status{2, "cooc_partition_plan must precede cooc_partition_pack"};
  if (d_row_nnz)
    COOC_HIP_TRY(hipMemcpyAsync(d_row_nnz, perm_nnz_.p, sizeof(int32_t) * M, hipMemcpyDeviceToDevice, s));
  if (d_entries && r.dense) {
    int dev = 0, n_cu = 256;
    COOC_HIP_TRY(hipGetDevice(&dev));
    COOC_HIP_TRY(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    k_pack_entries_dense<<<unsigned(std::max<int32_t>(1, std::min<int32_t>(M, 4 * n_cu))), kThreads, 0, s>>>(
        r.dense, perm_off_.as<int64_t>(), M, n_parts, d_entries);
    COOC_HIP_TRY(hipGetLastError());
  } else if (d_entries) {
    k_pack_entries<<<std::min<unsigned>(blocks_for(int64_t(M) * 64, 256), 8192), 256, 0, s>>>(
        r.row_base, r.row_nnz, r.col, r.cnt, perm_off_.as<int64_t>(), M, n_parts, d_entries);
    COOC_HIP_TRY(hipGetLastError());
  }
  return Status::Ok();
}

Status Sharder::merge(int32_t M, int32_t n_parts, int32_t part, const int32_t *d_recv_nnz, const uint64_t *d_entries,
                      const int64_t *d_rowsum_global, hipStream_t s, MergeResult *out) {
  if (part < 0 || part >= n_parts) return Status{1, "part outside [0, n_parts)"};
  const int32_t R = rows_owned(M, n_parts, part);
  const int64_t K = int64_t(n_parts) * R;
  COOC_TRY(recv_off_.reserve(sizeof(int64_t) * (K + 1)));
  COOC_TRY(cap_.reserve(sizeof(int64_t) * (R + 1)));
  COOC_TRY(row_base_.reserve(sizeof(int64_t) * (R + 1)));
  COOC_TRY(row_nnz_.reserve(sizeof(int32_t) * (R + 1)));
  COOC_TRY(rowsum_.reserve(sizeof(int64_t) * (R + 1)));
  COOC_TRY(err_.reserve(sizeof(int64_t) * 2));
  COOC_HIP_TRY(hipMemsetAsync(err_.p, 0, sizeof(int64_t) * 2, s));
  size_t b1 = 0, b2 = 0;
  hipcub::TransformInputIterator<int64_t, WidenI64, const int32_t *> recv64(d_recv_nnz, WidenI64{});
  COOC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, b1, recv64, recv_off_.as<int64_t>(), int(K), s));
  COOC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, b2, cap_.as<int64_t>(), row_base_.as<int64_t>(), R + 1, s));
  COOC_TRY(tmp_.reserve(std::max(b1, b2)));
  if (K > 0) {
    size_t b = tmp_.cap;
    COOC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp_.p, b, recv64, recv_off_.as<int64_t>(), int(K), s));
  }
  COOC_HIP_TRY(hipMemsetAsync(cap_.as<int64_t>() + R, 0, sizeof(int64_t), s));
  if (R > 0) k_merge_plan<<<blocks_for(R, 256), 256, 0, s>>>(d_recv_nnz, n_parts, R, M, cap_.as<int64_t>());
  {
    size_t b = tmp_.cap;
    COOC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp_.p, b, cap_.as<int64_t>(), row_base_.as<int64_t>(), R + 1, s));
  }
  int64_t cap_total = 0;
  COOC_HIP_TRY(hipMemcpyAsync(&cap_total, row_base_.as<int64_t>() + R, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  COOC_TRY(col_.reserve(sizeof(int32_t) * (cap_total + 1)));
  COOC_TRY(cnt_.reserve(sizeof(uint32_t) * (cap_total + 1)));
  if (R > 0 && int64_t(M) * 4 > kMergeDenseMaxBytes) {
    // a universe whose dense row does not fit the LDS: the received entries sorted by (owned row, column) and runs
    // of equal keys summed (library radix sort + reduce-by-key; the exchange path of streaming windows at p > 1)
    int64_t n_recv = 0;
    COOC_HIP_TRY(hipMemcpyAsync(&n_recv, recv_off_.as<int64_t>() + K - 1, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    int32_t last = 0;
    COOC_HIP_TRY(hipMemcpyAsync(&last, d_recv_nnz + K - 1, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    COOC_HIP_TRY(hipStreamSynchronize(s));
    n_recv += last;
    COOC_TRY(skeys_.reserve(sizeof(uint64_t) * size_t(2 * n_recv + 2)));
    COOC_TRY(svals_.reserve(sizeof(uint32_t) * size_t(2 * n_recv + 2) + sizeof(int64_t)));
    uint64_t *k0 = skeys_.as<uint64_t>(), *k1 = k0 + n_recv + 1;
    uint32_t *v0 = svals_.as<uint32_t>(), *v1 = v0 + n_recv + 1;
    int64_t *n_runs = reinterpret_cast<int64_t *>(svals_.as<char>() + sizeof(uint32_t) * size_t(2 * n_recv + 2));
    COOC_HIP_TRY(hipMemsetAsync(n_runs, 0, sizeof(int64_t), s));
    if (n_recv > 0) {
      k_merge_keys<<<std::min<unsigned>(blocks_for(K * 64, 256), 8192), 256, 0, s>>>(
          d_recv_nnz, recv_off_.as<int64_t>(), d_entries, K, R, k0, v0);
      int kb = 33;
      while ((int64_t(1) << (kb - 32)) < int64_t(R) && kb < 64) kb++;
      size_t bs = 0, br = 0;
      COOC_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, bs, k0, k1, v0, v1, int(n_recv), 0, kb, s));
      COOC_HIP_TRY(hipcub::DeviceReduce::ReduceByKey(nullptr, br, k1, k0, v1, v0, n_runs, hipcub::Sum(), int(n_recv), s));
      COOC_TRY(tmp_.reserve(std::max(bs, br)));
      bs = tmp_.cap;
      COOC_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp_.p, bs, k0, k1, v0, v1, int(n_recv), 0, kb, s));
      br = tmp_.cap;
      COOC_HIP_TRY(hipcub::DeviceReduce::ReduceByKey(tmp_.p, br, k1, k0, v1, v0, n_runs, hipcub::Sum(), int(n_recv), s));
    }
    k_merge_rows_from_keys<<<std::min<unsigned>(blocks_for(int64_t(R) * 64, 256), 8192), 256, 0, s>>>(
        k0, v0, n_runs, R, part, n_parts, row_base_.as<int64_t>(), row_nnz_.as<int32_t>(), col_.as<int32_t>(),
        cnt_.as<uint32_t>(), d_rowsum_global, rowsum_.as<int64_t>(), err_.as<int64_t>());
    COOC_HIP_TRY(hipGetLastError());
  } else if (R > 0) {
    const size_t lds = size_t(M) * 4;
    COOC_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(k_merge_rows),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
    int dev = 0, n_cu = 256;
    COOC_HIP_TRY(hipGetDevice(&dev));
    COOC_HIP_TRY(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    k_merge_rows<<<unsigned(std::min<int64_t>(R, n_cu)), kThreads, lds, s>>>(
        d_recv_nnz, recv_off_.as<int64_t>(), d_entries, n_parts, R, M, part, n_parts, row_base_.as<int64_t>(),
        row_nnz_.as<int32_t>(), col_.as<int32_t>(), cnt_.as<uint32_t>(), d_rowsum_global, rowsum_.as<int64_t>(),
        err_.as<int64_t>());
    COOC_HIP_TRY(hipGetLastError());
  }
  int64_t h_err = 0;
  COOC_HIP_TRY(hipMemcpyAsync(&h_err, err_.p, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  if (h_err & 2) return Status{5, "merged row sum differs from the all-reduced row sum (uint32 overflow)"};
  out->n_rows = R;
  out->row_base = row_base_.as<int64_t>();
  out->row_nnz = row_nnz_.as<int32_t>();
  out->col = col_.as<int32_t>();
  out->cnt = cnt_.as<uint32_t>();
  out->rowsum = rowsum_.as<int64_t>();
  return Status::Ok();
}

void Sharder::release() {
  DevBuf *all[] = {&perm_nnz_, &perm_off_, &part_entries_, &tmp_, &recv_off_, &cap_,
                   &row_base_, &row_nnz_, &col_, &cnt_, &rowsum_, &err_, &skeys_, &svals_};
  for (DevBuf *b : all) b->release();
}

}  // namespace cooc
