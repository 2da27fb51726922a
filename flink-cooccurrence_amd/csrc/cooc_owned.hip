// cooc_owned.hip — one window of the multi-GPU large-universe job inside the library (cooc_count_owned,
// cooc_topk_owned): the reference's keyBy(user) / keyBy(ItemCooccurrences::getItem) / broadcast()
// exchanges (FlinkCooccurrences.java:70,152,163) as collectives of the context's communicator
// (cooc_comm.h: RCCL over xGMI, or caller operations) around the owned-rows count of cooc_sparse.hip.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include "cooc_comm.h"
#include "cooc_ctx.h"
#include "cooc_scan.h"
#include "cooc_stream_kernels.h"

using cooc::Status;

namespace {

constexpr int32_t kSnakeHead = 4096;  // rows placed greedily (sharding.snake_owner's head)

__global__ void k_iota(int32_t *v, int32_t n) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = i;
}

// owner[order[i]]: the head's greedy ranks, then the snake over the ranks sorted by load
__global__ void k_owner_assign(const int32_t *__restrict__ order, int32_t M, int32_t h,
                               const int32_t *__restrict__ head_owner, const int32_t *__restrict__ rank_by_load,
                               int32_t world, int32_t *__restrict__ owner) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  int32_t o;
  if (i < h) {
    o = head_owner[i];
  } else {
    const int64_t pos = int64_t(i) - h, lap = pos / world, r = pos % world;
    o = rank_by_load[(lap & 1) == 0 ? r : world - 1 - r];
  }
  owner[order[i]] = o;
}

__global__ void k_lengths(const int64_t *__restrict__ up, int64_t U, int64_t *__restrict__ lens) {
  const int64_t j = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j < U) lens[j] = up[j + 1] - up[j];
}

inline unsigned nblk(int64_t n, int t) { return unsigned(std::max<int64_t>(1, (n + t - 1) / t)); }

int bits_needed(int64_t v) {
  int b = 1;
  while (b < 63 && (int64_t(1) << b) <= v) b++;
  return b;
}

}  // namespace

Status cooc_ctx::count_owned(int64_t n_users, const int64_t *d_up, const int32_t *d_items, int64_t n, hipStream_t s,
                             cooc_owned_info *info, cooc_device_result *out) {
  if (!comm) return Status{COOC_ERR_STATE, "cooc_count_owned needs a communicator (cooc_comm_init)"};
  if (!counter.sparse())
    return Status{COOC_ERR_ARG, "cooc_count_owned needs n_items >= " + std::to_string(cooc::Counter::kBatchMaxItems)};
  COOC_HIP_TRY(hipSetDevice(device));
  cooc::Comm &C = *comm;
  const int32_t M = cfg.n_items, W = C.world(), me = C.rank();
  // (1) global item frequencies
  COOC_TRY(own_counts.reserve(sizeof(int64_t) * size_t(M)));
  int64_t *counts = own_counts.as<int64_t>();
  COOC_TRY(cooc::launch_item_counts(s, d_items, n, M, counts));
  COOC_TRY(C.allreduce_sum_i64(counts, M, s));
  // (2) owner map: rows by descending frequency (a stable radix sort: ties keep the smaller id first)
  COOC_TRY(own_sort.reserve(sizeof(int64_t) * size_t(M) + 2 * sizeof(int32_t) * size_t(M)));
  int64_t *skeys = own_sort.as<int64_t>();
  int32_t *ids = reinterpret_cast<int32_t *>(skeys + M), *order = ids + M;
  k_iota<<<nblk(M, 256), 256, 0, s>>>(ids, M);
  size_t tmp = 0;
  const int kb = bits_needed(std::max<int64_t>(1, n) * std::max<int64_t>(1, W));  // counts < n_total <= W * max n
  COOC_HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tmp, counts, skeys, ids, order, M, 0, 64, s));
  COOC_TRY(own_tmp.reserve(tmp));
  (void)kb;  // (the global total is not known before the all-reduce: all 64 bits)
  COOC_HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(own_tmp.p, tmp, counts, skeys, ids, order, M, 0, 64, s));
  const int32_t h = std::min(kSnakeHead, M);
  std::vector<int64_t> head_counts(size_t(h) + 1);
  COOC_HIP_TRY(hipMemcpyAsync(head_counts.data(), skeys, sizeof(int64_t) * size_t(h), hipMemcpyDeviceToHost, s));
  // sizes of every rank's part, gathered in the same sync
  COOC_TRY(own_sizes.reserve(sizeof(int64_t) * size_t(2 + 2 * W)));
  int64_t *d_sz = own_sizes.as<int64_t>();
  const int64_t my_sz[2] = {n_users, n};
  COOC_HIP_TRY(hipMemcpyAsync(d_sz, my_sz, sizeof(my_sz), hipMemcpyHostToDevice, s));
  COOC_TRY(C.allgather(d_sz, d_sz + 2, 2 * sizeof(int64_t), s));
  std::vector<int64_t> sz(static_cast<size_t>(2 * W));
  COOC_HIP_TRY(hipMemcpyAsync(sz.data(), d_sz + 2, sizeof(int64_t) * size_t(2 * W), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  std::vector<int32_t> head_owner(size_t(h) + 1);
  std::vector<int32_t> rank_by_load(static_cast<size_t>(W));
  cooc::snake_head(head_counts.data(), h, W, head_owner.data(), rank_by_load.data());
  COOC_TRY(own_owner.reserve(sizeof(int32_t) * (size_t(M) + size_t(h) + size_t(W))));
  int32_t *owner = own_owner.as<int32_t>(), *d_head = owner + M, *d_rbl = d_head + h;
  COOC_HIP_TRY(hipMemcpyAsync(d_head, head_owner.data(), sizeof(int32_t) * size_t(h), hipMemcpyHostToDevice, s));
  COOC_HIP_TRY(hipMemcpyAsync(d_rbl, rank_by_load.data(), sizeof(int32_t) * size_t(W), hipMemcpyHostToDevice, s));
  k_owner_assign<<<nblk(M, 256), 256, 0, s>>>(order, M, h, d_head, d_rbl, W, owner);
  COOC_HIP_TRY(hipGetLastError());
  // (3) the histories, all-gathered into one compact CSR (parts in rank order)
  int64_t U_all = 0, N_all = 0;
  const size_t Wn = static_cast<size_t>(W);
  std::vector<int64_t> u_off(Wn), n_off(Wn), u_bytes(Wn), n_bytes(Wn);
  for (int32_t r = 0; r < W; r++) {
    u_off[size_t(r)] = U_all * int64_t(sizeof(int64_t));
    n_off[size_t(r)] = N_all * int64_t(sizeof(int32_t));
    u_bytes[size_t(r)] = sz[size_t(2 * r)] * int64_t(sizeof(int64_t));
    n_bytes[size_t(r)] = sz[size_t(2 * r + 1)] * int64_t(sizeof(int32_t));
    U_all += sz[size_t(2 * r)];
    N_all += sz[size_t(2 * r + 1)];
  }
  if (sz[size_t(2 * me)] != n_users || sz[size_t(2 * me + 1)] != n)
    return Status{COOC_ERR_STATE, "cooc_count_owned: the gathered sizes disagree with this rank's part"};
  COOC_TRY(own_lens.reserve(sizeof(int64_t) * size_t(std::max<int64_t>(1, n_users + U_all))));
  int64_t *lens = own_lens.as<int64_t>(), *lens_all = lens + n_users;
  COOC_TRY(own_up.reserve(sizeof(int64_t) * size_t(U_all + 1)));
  COOC_TRY(own_items.reserve(sizeof(int32_t) * size_t(std::max<int64_t>(1, N_all))));
  int64_t *up_all = own_up.as<int64_t>();
  int32_t *it_all = own_items.as<int32_t>();
  if (n_users > 0) k_lengths<<<nblk(n_users, 256), 256, 0, s>>>(d_up, n_users, lens);
  const std::vector<int64_t> zero(Wn, 0), my_u(Wn, n_users * int64_t(sizeof(int64_t))),
      my_n(Wn, n * int64_t(sizeof(int32_t)));
  // every rank sends its whole part to every peer (send offsets all 0); the parts land compact, in rank order
  COOC_TRY(C.alltoallv(lens, zero.data(), my_u.data(), lens_all, u_off.data(), u_bytes.data(), s));
  COOC_TRY(C.alltoallv(d_items, zero.data(), my_n.data(), it_all, n_off.data(), n_bytes.data(), s));
  COOC_HIP_TRY(hipMemsetAsync(up_all, 0, sizeof(int64_t), s));
  // the gathered lengths' prefix (cooc_scan.h; own_tmp holds the tile statuses and, after them, the error word)
  const int64_t scan_words = cooc::scan_state_words(std::max<int64_t>(U_all, 1));
  COOC_TRY(own_tmp.reserve(sizeof(unsigned long long) * size_t(scan_words + 1)));
  int64_t *scan_err = reinterpret_cast<int64_t *>(own_tmp.as<unsigned long long>() + scan_words);
  COOC_HIP_TRY(hipMemsetAsync(scan_err, 0, sizeof(int64_t), s));
  COOC_TRY(cooc::launch_scan<true>(cooc::ScanI64{lens_all}, up_all + 1, U_all, own_tmp.as<unsigned long long>(), scan_err, s));
  int64_t h_scan_err = 0;
  COOC_HIP_TRY(hipMemcpyAsync(&h_scan_err, scan_err, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  // (4) the owned rows over every user
  COOC_TRY(count_device_owned(U_all, up_all, it_all, N_all, owner, me, counts, N_all, s, out));
  // (5) the job's ordered pairs
  COOC_TRY(own_obs.reserve(sizeof(int64_t)));
  int64_t obs = out->observed;
  COOC_HIP_TRY(hipMemcpyAsync(own_obs.p, &obs, sizeof(int64_t), hipMemcpyHostToDevice, s));
  COOC_TRY(C.allreduce_sum_i64(own_obs.as<int64_t>(), 1, s));
  int64_t obs_all = 0;
  COOC_HIP_TRY(hipMemcpyAsync(&obs_all, own_obs.p, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  if (h_scan_err & 8) return Status{COOC_ERR_STATE, "internal bounds check failed (gathered history prefix)"};
  info->part = me;
  info->n_parts = W;
  info->observed = obs_all;
  info->local_observed = out->observed;
  info->n_users_all = U_all;
  info->n_interactions_all = N_all;
  info->gathered_bytes = int64_t(sizeof(int32_t)) * (N_all - n) + int64_t(sizeof(int64_t)) * (U_all - n_users);
  info->owner = owner;
  info->item_counts = counts;
  return Status::Ok();
}

Status cooc_ctx::topk_owned(int32_t topk, int32_t flags, int32_t *d_sizes, int32_t *d_values, double *d_scores,
                            int64_t *d_rowsum_global, hipStream_t s) {
  if (!comm) return Status{COOC_ERR_STATE, "cooc_topk_owned needs a communicator (cooc_comm_init)"};
  if (!have_batch) return Status{COOC_ERR_STATE, "no cooc_count_owned result on this context"};
  COOC_HIP_TRY(hipSetDevice(device));
  const int32_t M = cfg.n_items;
  COOC_TRY(own_rowsum.reserve(sizeof(int64_t) * size_t(M)));
  int64_t *rs = own_rowsum.as<int64_t>();
  COOC_HIP_TRY(hipMemcpyAsync(rs, batch_result.rowsum, sizeof(int64_t) * size_t(M), hipMemcpyDeviceToDevice, s));
  COOC_TRY(comm->allreduce_sum_i64(rs, M, s));
  if (d_rowsum_global)
    COOC_HIP_TRY(hipMemcpyAsync(d_rowsum_global, rs, sizeof(int64_t) * size_t(M), hipMemcpyDeviceToDevice, s));
  return topk_batch_device(topk, flags, rs, d_sizes, d_values, d_scores, s);
}
