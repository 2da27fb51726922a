// cooc_comm.cpp — RCCL (dlopen) and caller-operation transports of the multi-GPU exchange
// (cooc_comm.h).  Every collective is enqueued on the caller's HIP stream; nothing synchronises the
// device except where a host value is returned.
#include "cooc_comm.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <mutex>
#include <numeric>
#include <string>

namespace cooc {

namespace {

// The RCCL entry points the exchange uses, resolved once per process.  dlopen by soname: a process that
// already holds RCCL (torch links librccl.so.1) gets that same copy, a JVM gets /opt/rocm's.
struct Rccl {
  bool ok = false;
  std::string err;
  ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char *(*error_string)(ncclResult_t) = nullptr;
};

const Rccl &rccl_lib() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void *h = nullptr;
    for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (h) break;
    }
    if (!h) {
      const char *e = dlerror();
      r.err = std::string("RCCL is not available (dlopen librccl.so.1: ") + (e ? e : "?") + ")";
      return;
    }
    auto sym = [&](const char *n) { return dlsym(h, n); };
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(sym("ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(sym("ncclAllReduce"));
    r.all_gather = reinterpret_cast<decltype(r.all_gather)>(sym("ncclAllGather"));
    r.send = reinterpret_cast<decltype(r.send)>(sym("ncclSend"));
    r.recv = reinterpret_cast<decltype(r.recv)>(sym("ncclRecv"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
    r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_reduce && r.all_gather && r.send && r.recv &&
           r.group_start && r.group_end && r.error_string;
    if (!r.ok) r.err = "librccl.so.1 lacks an entry point the exchange needs";
  });
  return r;
}

Status nccl_status(ncclResult_t e, const char *what) {
  if (e == ncclSuccess) return Status::Ok();
  return Status{COOC_ERR_HIP, std::string(what) + ": " + rccl_lib().error_string(e)};
}

#define COOC_NCCL_TRY(expr, what)                  \
  do {                                             \
    ::cooc::Status s_ = nccl_status((expr), what); \
    if (!s_.ok()) return s_;                       \
  } while (0)

Status ops_status(int rc, const char *what) {
  if (rc == 0) return Status::Ok();
  return Status{COOC_ERR_STATE, std::string("cooc_comm_ops.") + what + " failed with " + std::to_string(rc)};
}

}  // namespace

Comm::~Comm() {
  if (comm_) (void)rccl_lib().comm_destroy(static_cast<ncclComm_t>(comm_));
}

Status Comm::unique_id(uint8_t *out) {
  const Rccl &r = rccl_lib();
  if (!r.ok) return Status{COOC_ERR_HIP, r.err};
  ncclUniqueId id;
  COOC_NCCL_TRY(r.get_unique_id(&id), "ncclGetUniqueId");
  std::copy(id.internal, id.internal + NCCL_UNIQUE_ID_BYTES, reinterpret_cast<char *>(out));
  return Status::Ok();
}

Status Comm::init_rccl(const uint8_t *unique_id, int32_t rank, int32_t world, int device) {
  const Rccl &r = rccl_lib();
  if (!r.ok) return Status{COOC_ERR_HIP, r.err};
  COOC_HIP_TRY(hipSetDevice(device));
  ncclUniqueId id;
  std::copy(unique_id, unique_id + NCCL_UNIQUE_ID_BYTES, reinterpret_cast<uint8_t *>(id.internal));
  ncclComm_t c = nullptr;
  COOC_NCCL_TRY(r.comm_init_rank(&c, world, id, rank), "ncclCommInitRank");
  comm_ = c;
  rank_ = rank;
  world_ = world;
  return Status::Ok();
}

Status Comm::init_ops(int32_t rank, int32_t world, const cooc_comm_ops &ops, void *user) {
  if (!ops.allreduce_sum_i64 || !ops.allgather || !ops.alltoallv)
    return Status{COOC_ERR_ARG, "cooc_comm_ops: every operation must be set"};
  ops_ = ops;
  user_ = user;
  have_ops_ = true;
  rank_ = rank;
  world_ = world;
  return Status::Ok();
}

Status Comm::allreduce_sum_i64(int64_t *d, int64_t n, hipStream_t s) {
  if (n <= 0) return Status::Ok();
  if (comm_)
    return nccl_status(rccl_lib().all_reduce(d, d, size_t(n), ncclInt64, ncclSum, static_cast<ncclComm_t>(comm_), s),
                       "ncclAllReduce");
  if (have_ops_) return ops_status(ops_.allreduce_sum_i64(user_, d, n, s), "allreduce_sum_i64");
  return Status{COOC_ERR_STATE, "no communicator (cooc_comm_init)"};
}

Status Comm::allgather(const void *d_send, void *d_recv, int64_t bytes, hipStream_t s) {
  if (comm_)
    return nccl_status(rccl_lib().all_gather(d_send, d_recv, size_t(bytes), ncclUint8, static_cast<ncclComm_t>(comm_), s),
                       "ncclAllGather");
  if (have_ops_) return ops_status(ops_.allgather(user_, d_send, d_recv, bytes, s), "allgather");
  return Status{COOC_ERR_STATE, "no communicator (cooc_comm_init)"};
}

Status Comm::alltoallv(const void *d_send, const int64_t *send_off, const int64_t *send_bytes, void *d_recv,
                       const int64_t *recv_off, const int64_t *recv_bytes, hipStream_t s) {
  if (comm_) {
    // every peer pair at once (one group): on xGMI each peer transfer has a link of its own; the rank's own
    // part is a device copy
    const Rccl &r = rccl_lib();
    const auto *src = static_cast<const uint8_t *>(d_send);
    auto *dst = static_cast<uint8_t *>(d_recv);
    if (send_bytes[rank_] != recv_bytes[rank_]) return Status{COOC_ERR_ARG, "alltoallv: self send != self receive"};
    if (send_bytes[rank_] > 0)
      COOC_HIP_TRY(hipMemcpyAsync(dst + recv_off[rank_], src + send_off[rank_], size_t(send_bytes[rank_]),
                                  hipMemcpyDeviceToDevice, s));
    COOC_NCCL_TRY(r.group_start(), "ncclGroupStart");
    for (int32_t p = 0; p < world_; p++) {
      if (p == rank_) continue;
      if (send_bytes[p] > 0)
        COOC_NCCL_TRY(r.send(src + send_off[p], size_t(send_bytes[p]), ncclUint8, p, static_cast<ncclComm_t>(comm_), s),
                      "ncclSend");
      if (recv_bytes[p] > 0)
        COOC_NCCL_TRY(r.recv(dst + recv_off[p], size_t(recv_bytes[p]), ncclUint8, p, static_cast<ncclComm_t>(comm_), s),
                      "ncclRecv");
    }
    COOC_NCCL_TRY(r.group_end(), "ncclGroupEnd");
    return Status::Ok();
  }
  if (have_ops_)
    return ops_status(ops_.alltoallv(user_, d_send, send_off, send_bytes, d_recv, recv_off, recv_bytes, s), "alltoallv");
  return Status{COOC_ERR_STATE, "no communicator (cooc_comm_init)"};
}

void snake_head(const int64_t *head_counts, int32_t h, int32_t world, int32_t *head_owner, int32_t *rank_by_load) {
  std::vector<int64_t> load(static_cast<size_t>(world), 0);
  for (int32_t i = 0; i < h; i++) {
    int32_t best = 0;  // least loaded rank, ties: the smaller rank (the (load, rank) min-heap of sharding.py)
    for (int32_t r = 1; r < world; r++)
      if (load[size_t(r)] < load[size_t(best)]) best = r;
    head_owner[i] = best;
    load[size_t(best)] += head_counts[i];
  }
  std::vector<int32_t> ord(static_cast<size_t>(world));
  std::iota(ord.begin(), ord.end(), 0);
  std::stable_sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return load[size_t(a)] < load[size_t(b)]; });
  std::copy(ord.begin(), ord.end(), rank_by_load);
}

void snake_owner_host(const int64_t *counts, int32_t M, int32_t world, int32_t head, int32_t *owner) {
  std::vector<int32_t> order(static_cast<size_t>(M));
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return counts[a] > counts[b]; });
  const int32_t h = std::min(head, M);
  std::vector<int64_t> hc(static_cast<size_t>(h));
  for (int32_t i = 0; i < h; i++) hc[size_t(i)] = counts[order[size_t(i)]];
  std::vector<int32_t> ho(static_cast<size_t>(h)), rbl(static_cast<size_t>(world));
  snake_head(hc.data(), h, world, ho.data(), rbl.data());
  for (int32_t i = 0; i < h; i++) owner[order[size_t(i)]] = ho[size_t(i)];
  for (int64_t pos = 0; pos < int64_t(M) - h; pos++) {
    const int64_t lap = pos / world, r = pos % world;
    owner[order[size_t(h + pos)]] = rbl[size_t(lap % 2 == 0 ? r : world - 1 - r)];
  }
}

}  // namespace cooc
