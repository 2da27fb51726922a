// cooc_stream_kernels.h — launch wrappers of cooc_stream.hip (resident streaming state).
#pragma once

#include "cooc_device.h"

namespace cooc {

Status launch_relocate(hipStream_t s, int64_t n, const int64_t *reloc, int32_t *arena);
// LogLikelihood.logLikelihoodRatio (the rescorer's device scoring function) over n (k11, k12, k21, k22)
Status launch_llr(hipStream_t s, int64_t n, const int64_t *d_k4, double *d_out);
// list j of len[j] ids at arena offset off[j] -> out[dst[j] ..) (contiguous CSR of arena slabs)
Status launch_gather_lists(hipStream_t s, int64_t n, const int64_t *off, const int32_t *len, const int64_t *dst,
                           const int32_t *arena, int32_t *out);
Status launch_append(hipStream_t s, int64_t n, const int64_t *new_ptr, const int64_t *new_dst, const int32_t *items,
                     int32_t *arena);
// scal: [0] touched rows, [1] sum of the window's int row-sum deltas, [2] rescorer observed
// (cumulative), [3] exact observed (cumulative).
Status launch_merge_global(hipStream_t s, int32_t M, const int64_t *row_base, const int32_t *row_nnz,
                           const int32_t *col, const uint32_t *cnt, const int64_t *rowsum_delta, uint32_t *G,
                           int64_t *grs, int64_t *scal, int64_t observed_window);
// p > 1 windows: the owner's merged rows (R rows a = part + r W) as an M-row view (base, nnz: zero elsewhere);
// their entries merged into the dense global rows G and every item's all-reduced row-sum delta rs_all into grs
// (scal[1]: sum of the int views over all items, scal[4]: over the owned rows with a delta); the view packed for
// copy-out (rp int64[M+1], *total entries; synchronises s).
Status launch_owned_view(hipStream_t s, int32_t M, int32_t W, int32_t part, int32_t R, const int64_t *mbase,
                         const int32_t *mnnz, int64_t *base, int32_t *nnz);
Status launch_merge_owned(hipStream_t s, int32_t M, const int64_t *base, const int32_t *nnz, const int32_t *col,
                          const uint32_t *cnt, const int64_t *rs_all, uint32_t *G, int64_t *grs, int64_t *scal,
                          int64_t observed_window);
Status launch_pack_rows(hipStream_t s, int32_t M, const int64_t *base, const int32_t *nnz, const int32_t *col,
                        const uint32_t *cnt, DevBuf &rp, DevBuf &out_col, DevBuf &out_cnt, DevBuf &tmp, int64_t *total);
// kMax cap of a device CSR: cut_ptr int64[n_users+1], cut_items int32[<= n]; *n_cut = cut_ptr[n_users]
// (read back: the caller sizes the next pass with it).
Status launch_user_cut(hipStream_t s, int64_t n_users, const int64_t *up, const int32_t *items, int32_t cut,
                       int64_t *cut_ptr, int32_t *cut_items, DevBuf &tmp, int64_t *n_cut);
Status launch_touched(hipStream_t s, int32_t M, const int32_t *row_nnz, int32_t *touched, int64_t *n_touched,
                      DevBuf &tmp);
size_t rescore_lds_bytes(int32_t topk);
Status launch_rescore(hipStream_t s, const int32_t *touched, const int64_t *scal, int32_t M, const uint32_t *G,
                      const int64_t *grs, bool exact, int32_t topk, int32_t max_rows, DevBuf &terms, int32_t *out_size,
                      int32_t *out_val, double *out_score);

// LLR top-k of every row of a batch result (padded CSR) -- the C5 stage over one window.
// obs3 (device int64[3]) receives the rescorer's observed, the exact observed and n_items; terms is
// scratch for the per-column LLR terms (32 B per item).
Status launch_rescore_batch(hipStream_t s, int32_t M, const int64_t *row_base, const int32_t *row_nnz,
                            const int32_t *col, const uint32_t *cnt, const uint32_t *dense, const int64_t *rowsum,
                            bool exact, int32_t topk,
                            int64_t *obs3, DevBuf &terms, int32_t *out_size, int32_t *out_val, double *out_score,
                            const int32_t *rank_of = nullptr, bool unordered = true, int64_t nnz = -1,
                            bool whole_log = false);

// Sparse global rows (n_items >= 40,320; the rescorer's itemRows, ItemRowRescorer...java:35,171-177):
// row a = len[a] (column, count) entries in ascending column order at base[a] of the arena (col, cnt).
// Rows move to a new bump-allocated slab when a window touches them; live = entries of all rows;
// the arena is compacted (rows re-laid in order) when a window would not fit behind the bump
// (struct GlobalSparse, cooc_device.h).
// Merge a window's packed delta rows (drp int64[M+1], dcol, dcnt; nnz entries) into the rows;
// *new_cols = the window's new (row, column) keys.  Synchronises the stream.
Status launch_gs_merge(hipStream_t s, int32_t M, const int64_t *drp, const int32_t *dcol, const uint32_t *dcnt,
                       int64_t nnz, GlobalSparse &g, DevBuf &tmp, int64_t *new_cols);
Status compact_global(hipStream_t s, int32_t M, GlobalSparse &g, DevBuf &tmp, int64_t new_cap);
Status launch_rescore_sparse(hipStream_t s, const int32_t *touched, const int64_t *scal, int32_t M, const GlobalSparse &g,
                             const int64_t *grs, bool exact, int32_t topk, int32_t max_rows, DevBuf &terms,
                             int32_t *out_size, int32_t *out_val, double *out_score);

}  // namespace cooc
