// cooc_comm.h — the multi-GPU transport behind cooc_comm_init* (include/cooc.h): the reference's
// keyed exchanges (keyBy(user) FlinkCooccurrences.java:70, keyBy(ItemCooccurrences::getItem) :152,
// rowSumStream.broadcast() :163) as collectives on one context's HIP stream.
//
// Two transports behind one interface:
//   * RCCL over xGMI (the product path): librccl.so.1 is resolved with dlopen at cooc_comm_init time,
//     so the library loads (and its CPU tests run) where RCCL is absent, and a process that already
//     loaded RCCL (torch) shares that copy (same soname);
//   * caller operations (cooc_comm_ops): the same orchestration over any collective library the caller
//     has (the 2-process gloo tests drive the library's exchange through torch.distributed with it).
#pragma once

#include <cstdint>
#include <vector>

#include "../../include/cooc.h"
#include "cooc_device.h"

namespace cooc {

class Comm {
 public:
  ~Comm();
  Status init_rccl(const uint8_t *unique_id, int32_t rank, int32_t world, int device);
  Status init_ops(int32_t rank, int32_t world, const cooc_comm_ops &ops, void *user);
  int32_t rank() const { return rank_; }
  int32_t world() const { return world_; }
  bool rccl() const { return comm_ != nullptr; }

  // in-place sum over the ranks of an int64 device array, on stream s
  Status allreduce_sum_i64(int64_t *d, int64_t n, hipStream_t s);
  // every rank's `bytes` at d_send land at d_recv + r * bytes (rank order)
  Status allgather(const void *d_send, void *d_recv, int64_t bytes, hipStream_t s);
  // uneven exchange: send_bytes[p] bytes from d_send + send_off[p] go to rank p, which receives them at
  // its d_recv + recv_off[me]; recv_bytes[p] bytes arrive from rank p (all host arrays of world entries)
  Status alltoallv(const void *d_send, const int64_t *send_off, const int64_t *send_bytes, void *d_recv,
                   const int64_t *recv_off, const int64_t *recv_bytes, hipStream_t s);

  static Status unique_id(uint8_t *out);

 private:
  int32_t rank_ = 0, world_ = 1;
  void *comm_ = nullptr;  // ncclComm_t (RCCL transport)
  bool have_ops_ = false;
  cooc_comm_ops ops_{};
  void *user_ = nullptr;
};

// The row owner map of the multi-GPU large-universe exchange (sharding.snake_owner restated): rows
// sorted by descending global frequency (ties: smaller id first); the `head` most frequent are placed
// greedily on the least loaded rank (load = summed frequency, ties: smaller rank), the rest dealt in
// snake order over the ranks sorted by that load.  Host version over host counts (tests, JVM callers).
void snake_owner_host(const int64_t *counts, int32_t M, int32_t world, int32_t head, int32_t *owner);
// The greedy head placement shared by the host and device versions: head_counts (descending) -> the
// head's ranks and the ranks ordered by final load (rank_by_load[world]).
void snake_head(const int64_t *head_counts, int32_t h, int32_t world, int32_t *head_owner, int32_t *rank_by_load);

}  // namespace cooc
