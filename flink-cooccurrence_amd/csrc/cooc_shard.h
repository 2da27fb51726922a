// cooc_shard.h — owner-partitioned exchange of partial rows (cooc_shard.hip).
#pragma once

#include "cooc_device.h"

namespace cooc {

struct MergeResult {
  int32_t n_rows = 0;  // rows owned: a = part + r * n_parts
  int64_t *row_base = nullptr;
  int32_t *row_nnz = nullptr;
  int32_t *col = nullptr;
  uint32_t *cnt = nullptr;
  int64_t *rowsum = nullptr;
};

// Owned rows are merged in one dense LDS row of n_items counters up to this many bytes, by sorting above it.
constexpr int64_t kMergeDenseMaxBytes = 160 * 1024 - 1024;

class Sharder {
 public:
  // Entries of the last local result destined to every owner (host array of n_parts).
  Status plan(const CountResult &r, int32_t M, int32_t n_parts, hipStream_t s, int64_t *h_entries);
  // Row lengths in (owner, row) order and packed (col << 32 | cnt) entries in the same order.
  Status pack(const CountResult &r, int32_t M, int32_t n_parts, hipStream_t s, int32_t *d_row_nnz,
              uint64_t *d_entries);
  // Merge the partial rows received from n_parts sources (source-major buffers).
  Status merge(int32_t M, int32_t n_parts, int32_t part, const int32_t *d_recv_nnz, const uint64_t *d_entries,
               const int64_t *d_rowsum_global, hipStream_t s, MergeResult *out);
  void release();
  ~Sharder() { release(); }

 private:
  int32_t planned_parts_ = 0;
  DevBuf perm_nnz_, perm_off_, part_entries_, tmp_, recv_off_, cap_, row_base_, row_nnz_, col_, cnt_, rowsum_, err_;
  DevBuf skeys_, svals_;  // large universes: the received entries' sort keys and counts (merge)
};

}  // namespace cooc
