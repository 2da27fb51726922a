// cooc_sparse.hip — one window over empty histories for LARGE item universes (n_items >= 40,320,
// the C3 / C5 configs: 1e6 items), on gfx950.
//
// Same semantics as the batch path (cooc_count.hip): NonSampledUserInteractionCounter...java:113-165
// expanded from empty histories, reduced per row like ItemRowAggregator.java:26-31
// (Int2ShortOpenHashMap.addTo, exact uint32 here) and RowSumAggregator.java:25-27:
//   C[a, b] = sum_u #{ordered position pairs (p != q) : x_p = a, x_q = b},  rowsum[a] = sum_b C[a, b].
// A row a is the sum of the lists of the users that hold a (one "contribution" per interaction
// (u, a)), minus 1 at column a per contribution (the pair of a position with itself).
//
// At n_items = 1e6 a row cannot live in one LDS row (160 KB = 40K counters), and most rows are
// sparse: under Zipf(1) the row of an item of rank r holds ~W_1 / r pairs over up to 1e6 columns.
// The work unit is therefore a whole ROW, taken by one persistent workgroup per CU (heaviest rows
// first), which walks the row's column range as a sequence of CHUNKS and appends each chunk's
// entries, in column order, to the row's contiguous output (no gather pass):
//   * hash chunk  — a range of column tiles whose expected distinct keys fit an LDS open-addressing
//                   table (keys + counts, 1K..16K slots, the Int2ShortOpenHashMap of
//                   ItemRowAggregator.java:21-31 in LDS).  Sorted output without a sort: the keys'
//                   32-column blocks are ranked through a bitmap (L1) and per-block 32-bit masks, and
//                   an entry's slot is its block's base + the popcount of its mask below it.  A table
//                   that overflows (more distinct keys than expected) is redone with a 4x table, and
//                   at 16K slots as dense tiles.
//   * dense chunk — one column tile of 32,768 columns as uint32 LDS counters (one ds_add per pair),
//                   compacted in column order.
// The chunk plan of a row comes from its pair work W_a (exact) and the expected distinct keys per
// tile, E[d_t | W] = sum_{b in t} 1 - exp(-W f_b / N) (f_b = global frequency of b), tabulated per
// tile for W = 2^(k/2).  Per-user lists are regrouped by tile once (tb[u][t] = first position of
// tile t in u's list), so a tile range of a user's list is one contiguous segment.
// The few rows above kSplitWork pairs (the hottest items) are split into (row, tile, contribution
// range) work items that add into a dense uint32 staging row in HBM; a finalize kernel compacts
// each staging row (with the uint32 overflow check: sum of the counts == the closed-form row sum).
//
// HBM layout: tarena uint32[N] (tile-grouped user lists), tb int32[U x (T+1)], contributions
// (item-sorted user indices) uint32[N], epre int64[N+1] (prefix of the contributions' list
// lengths), per-row plan (W, two 64-bit tile masks), output = padded CSR (row_base, row_nnz, col,
// cnt) over per-workgroup slabs of a bump-allocated region.
#include <hipcub/hipcub.hpp>

#include "cooc_device.h"
#include "cooc_scan.h"
#include "cooc_radix.h"
#include <cstdio>
#include <cstring>
#include <vector>
#include <unistd.h>
#ifdef COOC_SP_STATS
#define STAT_CLOCK() wall_clock64()
#define STAT_ADD(k, v) do { if (threadIdx.x == 0) S_.st[k] += (v); } while (0)  // LDS: keeps occupancy
#else
#define STAT_CLOCK() 0ull
#define STAT_ADD(k, v) do {} while (0)
#endif
#ifdef COOC_SP_STATS
#define SRB_STAT(k, v) do { if (threadIdx.x == 0) atomicAdd(srb_st + (k), (unsigned long long)(v)); } while (0)
#else
#define SRB_STAT(k, v) do {} while (0)
#endif
#ifdef COOC_SP_TRACE
#define SPT(msg) do { hipStreamSynchronize(s); fprintf(stderr, "[sp] %s\n", msg); } while (0)
#else
#define SPT(msg) do {} while (0)
#endif

namespace cooc {

namespace {

#ifndef COOC_SP_THREADS
#define COOC_SP_THREADS 512
#endif
#ifndef COOC_SP_TSHIFT
#define COOC_SP_TSHIFT 14
#endif
constexpr int kSpThreads = COOC_SP_THREADS;  // 512: two workgroups per CU
constexpr int kSpWaves = kSpThreads / 64;
constexpr int kTShift = COOC_SP_TSHIFT;
constexpr int kTW = 1 << kTShift;  // dense tile width (16384: 64 KB of uint32 LDS counters)
constexpr int kSpMaxTiles = 64;                        // per-row plans are 64-bit tile masks
constexpr uint64_t kGatherFlag = 1;                    // in a row plan's hz[0] (tile 0's code slot, tile 0 dense)
constexpr int kHashMax = 8192;                        // slots: keys + counts = the dense tile's 128 KB
constexpr int kWStage = kHashMax / 2;                  // hash compaction: entries staged in LDS for 16-B stores
constexpr int kHashMin = 1024;                         // one slot per thread at least
constexpr int kHashMaxTiles = (1 << 20) / kTW;          // a hash chunk spans <= 2^20 columns ...
constexpr int kL1Words = kHashMaxTiles * kTW / 1024;   // ... so its block bitmap is <= 1024 words
constexpr int kSpDb = 512;                             // contribution descriptors per batch
constexpr int kMaxProbe = 64;                          // linear probes before an insert gives up
constexpr int kSpU = 4;                                // partner loads in flight per lane
constexpr int kEstK = 84;                              // estimate table: W_k = 2^(k/2), k < kEstK
constexpr int kTinyW = 256;                            // rows of at most this many pairs: one wave each (k_sp_tiny)
constexpr int kSmallW = 4096;                          // ... of at most this many: one 512-thread workgroup each (k_sp_small)
#ifndef COOC_SP_SPLIT_LG
#define COOC_SP_SPLIT_LG 23
#endif
#ifndef COOC_SP_GATHER_MIN
#define COOC_SP_GATHER_MIN 4  // rows of >= 4 chunks gather (A/B at round-4 HEAD: 125.2-125.5 vs 127.3-127.4 ms with 3)
#endif
constexpr int64_t kSplitWork = int64_t(1) << COOC_SP_SPLIT_LG;  // rows above this pair work are split
#ifndef COOC_SP_SUB_LG
#define COOC_SP_SUB_LG 24  // 2^24-pair shares: 1.4% faster than 2^23 on the 1/8 C3 shard (profiles/r03/sub_ab)
#endif
constexpr int64_t kSubWork = int64_t(1) << COOC_SP_SUB_LG;  // pairs per split work item (expected)
constexpr int64_t kScrGroups = int64_t(1) << 21;       // gather scratch per workgroup (16-B groups of 4 ids)
constexpr int kGatherMinChunks = COOC_SP_GATHER_MIN;   // rows with this many chunks gather their tails
#ifndef COOC_SP_FILL
#define COOC_SP_FILL 0.45f  // A/B at C3 (round 4, small rows in k_sp_small): 0.45 126.7, 0.5 126.9 (a row overflows), 0.375 130.3, 0.55 133 ms
#endif
#ifndef COOC_SP_DENSE
#define COOC_SP_DENSE 2.f
#endif
constexpr float kHashFill = COOC_SP_FILL * kHashMax;     // expected distinct keys per hash chunk
constexpr float kDensePairs = COOC_SP_DENSE * kTW;       // a tile with more expected pairs is dense
constexpr int kSpLds = kTW * 4 + 2 * kL1Words * 4 + kSpDb * 8 + (kSpDb + 4) * 4 + kSpThreads;  // (gb + info: 8 B per descriptor)

// Two shapes of the accumulate kernel, one queue.  Rows of at most kMidW pairs ("mid rows": at C3 the half
// million rows of 4K..64K pairs, mostly one dense tile 0 plus a sparse tail) run with FOUR 256-thread
// workgroups per CU instead of two 512-thread ones: their chunks are short latency chains (walk, barrier,
// compaction), so more independent chunks per CU hide more of them.  The LDS budget (40 KB per workgroup)
// holds because a count never exceeds its row's pair work W <= 65,535: the dense tile's counters are u16,
// two per LDS word (a ds_add of 1 << 16 for the odd column never carries), and hash tables have 4K slots
// (chunks of half the expected keys) over column spans of at most 2^19 (a 512-word block bitmap).
#ifndef COOC_SP_MID_W
#define COOC_SP_MID_W 65535
#endif
constexpr int64_t kMidW = COOC_SP_MID_W;
static_assert(kMidW <= 65535, "mid rows count in u16");
template <int Threads, int HashMax, int L1Words, int Db, bool U16>
struct SpShape {
  static constexpr int kThreads = Threads, kWaves = Threads / 64;
  static constexpr int kHashMax = HashMax;            // hash slots: keys [0, H) + counts [HashMax, HashMax + H)
  static constexpr int kWStage = HashMax / 2;         // compaction staging (entries) in the emptied table
  static constexpr int kL1Words = L1Words;            // block bitmap words: chunk spans <= L1Words * 1024 columns
  static constexpr int kHashMaxTiles = L1Words * 1024 / kTW;
  static constexpr int kDb = Db;                      // contribution descriptors per walk batch
  static constexpr bool kU16 = U16;                   // dense counters: u16 pairs (true) or u32
  static constexpr int kPer = U16 ? 8 : 4;            // dense counters per 16-B LDS word
  static constexpr int kRWords = (U16 ? kTW / 2 : kTW) > 2 * HashMax ? (U16 ? kTW / 2 : kTW) : 2 * HashMax;
  static constexpr int kLds = kRWords * 4 + 2 * L1Words * 4 + Db * 8 + (Db + 4) * 4 + Threads;
};
using SpBig = SpShape<kSpThreads, kHashMax, kL1Words, kSpDb, false>;
using SpMid = SpShape<256, 4096, 512, 256, true>;  // 40.9 KB of LDS: three per CU (four at 38.9 KB with 2^18-column spans measured slower: more chunks)
static_assert(SpBig::kLds == kSpLds, "the big shape is the original kernel");
constexpr float kHashFillMid = COOC_SP_FILL * SpMid::kHashMax;
// a tile whose expected distinct keys exceed this is a dense chunk (its own tile of counters, compacted by a
// linear sweep) rather than part of a hash chunk (A/B knobs; default: the hash chunk's own capacity)
#ifndef COOC_SP_BIG_DENSE
#define COOC_SP_BIG_DENSE kHashFill
#endif
#ifndef COOC_SP_MID_DENSE
#define COOC_SP_MID_DENSE kHashFillMid
#endif
constexpr float kDenseKeys = COOC_SP_BIG_DENSE, kDenseKeysMid = COOC_SP_MID_DENSE;

// One work item of k_sp_main, everything its start needs in one 64-B record (k_sp_queue).
struct SpWork {
  int64_t k0, k1;   // contribution range (row-sorted)
  uint64_t st, dn;  // chunk plan: bit t of st = a chunk starts at tile t, of dn = tile t is dense
  uint64_t hz[2];   // 2 bits per chunk-start tile: its hash table has kHashMin << code slots
  int32_t row;
  int32_t kind;     // -1: a whole row; -2: a share of a split row (every tile, into its staging row)
  int32_t gslot;    // >= 0: the item runs in gather mode (its tails go through buckets)
  int32_t est;      // a whole row's expected keys (planner estimate; sizes its output region)
};

struct SpArgs {
  const SpWork *queue;
  PlanTotals *tot;
  int32_t *qctr;            // this launch's work counter (k_sp_main: the queue range [q_begin, q_end))
  int64_t q_begin, q_end;
  const uint32_t *vals;     // contributions: user index, item-sorted
  const int32_t *tb;        // [U x (T + 2)] a user's tile-0 range in arena0, its tile starts in arena1
  const uint4 *tarena;      // arena1: the lists' ids of tiles >= 1 (u32), in 16-B groups
  const uint4 *tarena0;     // arena0: the lists' tile-0 ids (u16), in 16-B groups
  const int64_t *epre;      // [n_contrib + 1] prefix of the contributions' list lengths (pair work)
  const float *gmass;       // [T] share of the interactions in each tile
  uint32_t *staging;        // [n_split x sstride]
  int64_t sstride;          // staging row stride: M rounded up to 4 (16-B aligned rows)
  const int32_t *split_slot;
  int32_t *col_out;
  uint32_t *cnt_out;
  unsigned long long *bump;
  int64_t cap;
  int64_t slab;
  int64_t *row_base;
  int32_t *row_nnz;
  int32_t M, T;
  unsigned long long *prog;   // COOC_SP_TRACE: per-workgroup progress in pinned host memory
  unsigned long long *stats;  // COOC_SP_STATS: per-phase clocks and counts
  int32_t exp;                // COOC_SP_STATS only: experiment selector (COOC_SP_EXP; results invalid when set)
  int64_t n_contrib, n_users, n_groups, n_groups0;
  uint4 *scratch;           // gather mode: per-workgroup tail buckets, scr_cap groups each
  int64_t scr_cap;          // 0: gather mode off
  const int64_t *rowsum;    // [M] closed-form row sums W_a - c_a (k_sp_plan): every whole row is checked
  const int64_t *spre;      // streaming window: [n_contrib + 1] prefix of the kSelfBit flags; NULL: all set
  int32_t *deferred;        // [M] whole rows left to the sort + segmented-reduce path (k_sr_*), in tot->n_deferred
  int32_t sort_all;         // COOC_FLAG_SORT_ROWS: every whole row goes to that path (A/B and tests)
  int32_t any_order;        // COOC_FLAG_ANY_ORDER: hash chunks emitted in slot order (no column ranking)
  // column relabel (batch windows, k_relabel_*): the kernels work in relabelled column space -- tile 0 holds
  // the batch's kTW most frequent items (hot_col[c], ascending ids), column c >= kTW the item c - kTW (its
  // own id shifted one tile up; the hot items leave holes there) -- and write the item ids to the output.
  // NULL: identity (streaming windows, and universes of at most one tile).
  const int32_t *hot_col;   // [kTW] column < kTW -> item id
  const int32_t *pos_of;    // [M] item id -> column
};

// the item of relabelled column r: a table lookup in tile 0 (64 KB, cache resident), arithmetic above it
__device__ inline int32_t relabel_col(const int32_t *hot_col, uint32_t r) {
  if (!hot_col) return int32_t(r);
  return r < uint32_t(kTW) ? hot_col[r] : int32_t(r) - kTW;
}
__device__ inline int32_t relabel_pos(const int32_t *pos_of, uint32_t a) { return pos_of ? pos_of[a] : int32_t(a); }
__device__ inline int32_t sp_col(const SpArgs &A, uint32_t r) { return relabel_col(A.hot_col, r); }
__device__ inline int32_t sp_rank(const SpArgs &A, int32_t a) { return relabel_pos(A.pos_of, uint32_t(a)); }

#ifdef COOC_SP_TRACE
#define PROG(A, k, v) do { if (threadIdx.x == 0) __hip_atomic_store((A).prog + blockIdx.x * 64 + (k), (unsigned long long)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); } while (0)
#define WPROG(A, v) do { if ((threadIdx.x & 63) == 0) __hip_atomic_store((A).prog + blockIdx.x * 64 + 16 + (threadIdx.x >> 6), (unsigned long long)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); } while (0)
#define BCHK(A, cond, bit) ((cond) ? true : (atomicOr((A).prog + 2047, (unsigned long long)(bit)), false))
#define TR(A, v) do { if (threadIdx.x == 0 || threadIdx.x == 64) { unsigned long long *q_ = (A).prog + 1024 + (threadIdx.x ? 512 : 0); unsigned long long n_ = __hip_atomic_load(q_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); __hip_atomic_store(q_ + 1 + (n_ & 255), (unsigned long long)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); __hip_atomic_store(q_, n_ + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); } } while (0)
#else
#define TR(A, v) do {} while (0)
#define BCHK(A, cond, bit) true
#define PROG(A, k, v) do {} while (0)
#define WPROG(A, v) do {} while (0)
#endif

// Bounds checks of the global index math (COOC_SP_CHECK builds, for fault hunting): a failed check sets err
// bit 8 (COOC_ERR_STATE "internal bounds check") and skips the access; release builds compile them out.
#ifdef COOC_SP_CHECK
#define SP_CHECK(A, cond) ((cond) ? true : (atomicOr(reinterpret_cast<unsigned long long *>(&(A).tot->err), 8ull), false))
#else
#define SP_CHECK(A, cond) true
#endif

// Values every thread of the workgroup holds identically (read from LDS after a barrier): made
// explicitly uniform so that the branches on them are scalar and no barrier sits in exec-masked code.
__device__ inline uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ inline int32_t uni(int32_t v) { return int32_t(__builtin_amdgcn_readfirstlane(uint32_t(v))); }
// (readfirstlane returns an int: each half goes through uint32_t, or a low half >= 2^31 would
// sign-extend over the high half -- output positions >= 2^31 came out negative and their rows unwritten)
__device__ inline int64_t uni(int64_t v) {
  const uint64_t u = uint64_t(v);
  const uint32_t hi = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(u >> 32)));
  const uint32_t lo = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(u)));
  return int64_t((uint64_t(hi) << 32) | uint64_t(lo));
}

__device__ inline uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// Block-wide exclusive scan (kWaves waves); *total = the block sum.  Two barriers.
template <int kWaves>
__device__ inline uint32_t block_excl_scan(uint32_t x, uint32_t *total, uint32_t *s_wtot) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan(x);
  if (lane == 63) s_wtot[wave] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kWaves; w++) {
    const uint32_t v = s_wtot[w];
    pre += w < wave ? v : 0u;
    tot += v;
  }
  __syncthreads();
  *total = uni(tot);
  return pre + inc - x;
}

__device__ inline uint64_t block_sum_u64(uint64_t v, uint64_t *s_red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) s_red[wave] = v;
  __syncthreads();
  uint64_t t = 0;
#pragma unroll
  for (int w = 0; w < kSpWaves; w++) t += s_red[w];
  __syncthreads();
  return t;
}

// E[distinct keys of tile t | pair work W], interpolated in log2(W) between table points.
__device__ inline float est_distinct(const float *est, int t, int64_t W) {
  if (W <= 0) return 0.f;
  const float x = 2.f * log2f(float(W));
  int k = int(x);
  if (k >= kEstK - 1) return est[t * kEstK + kEstK - 1];
  const float f = x - float(k);
  const float lo = est[t * kEstK + k], hi = est[t * kEstK + k + 1];
  return lo + f * (hi - lo);
}

// Work items of a split row: shares of about kSubWork pairs whose expected tails (the pairs outside
// tile 0, mass 1 - g0) fit a gather scratch.
__device__ inline int32_t sp_split_shares(int64_t W, float g0) {
  const float tail = float(W) * fmaxf(0.f, 1.f - g0);
  return max(int32_t((W + kSubWork - 1) / kSubWork), int32_t(ceilf(tail / float(3 * kScrGroups))));
}

// ---- planner kernels ------------------------------------------------------------------------------
// Two arenas hold the users' lists, tile by tile: tile 0 (columns < 16,384: the Zipf head, ~70% of the
// ids) as u16 ids in arena0 (8 ids per 16-B load; at C3 the 1/8 shard's tile-0 part is ~180 MB and stays
// in the Infinity Cache), tiles >= 1 as u32 ids in arena1, ids of one tile contiguous, no padding between
// tiles.  tb[u] has T + 2 entries: tb[u][0] / tb[u][T + 1] = start / end of u's tile-0 ids in arena0
// (u16 positions), tb[u][t] (1 <= t <= T) = the arena1 position of tile t's first id (tb[u][T] = the end
// of u's list there).  A chunk reads a tile range of a list as the 16-B groups covering it and masks the
// ids outside it by position.
constexpr uint32_t kSink = 0xFFFFFFFFu;
constexpr uint32_t kSink16 = 0xFFFFu;  // (arena0 pads; never a tile-0 id)

__device__ inline bool bit_of(const uint32_t *__restrict__ bits, uint32_t i) { return (bits[i >> 5] >> (i & 31u)) & 1u; }

// An id's column after the relabel: a hot id's position in tile 0 (pos_of, gathered), any other id + kTW
// (arithmetic); without a relabel the id itself.
__device__ inline int32_t planner_rank(const int32_t *__restrict__ pos_of, const uint32_t *__restrict__ hotbm, uint32_t it) {
  if (!pos_of) return int32_t(it);
  return bit_of(hotbm, it) ? pos_of[it] : int32_t(it) + kTW;
}

// The arenas' user regions, packed and dense: one wave per user counts its tile-0 ids (ballots) and
// writes len[j] = round8(tile-0 ids) << 32 | round4(other ids); their inclusive prefix (one scan) gives
// every user's base in arena0 (high half) and arena1 (low half).
__global__ __launch_bounds__(256) void k_sp_tile_counts(int64_t U, const int64_t *__restrict__ up,
                                                        const int32_t *__restrict__ items, int32_t M,
                                                        uint64_t *__restrict__ len, const int32_t *__restrict__ owner,
                                                        int32_t part, int32_t *__restrict__ ownc,
                                                        const int32_t *__restrict__ rank_of,
                                                        const uint32_t *__restrict__ hotbm,
                                                        const uint32_t *__restrict__ minebm) {
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t j = gw; j < U; j += n_waves) {
    const int64_t s = up[j];
    const int32_t n = int32_t(up[j + 1] - s);
    int32_t n0 = 0, mine = 0;
    for (int32_t p0 = 0; p0 < n; p0 += 4 * 64) {
      int32_t it[4];
#pragma unroll
      for (int k = 0; k < 4; k++) it[k] = p0 + 64 * k + lane < n ? items[s + p0 + 64 * k + lane] : -1;
#pragma unroll
      for (int k = 0; k < 4; k++) {  // (an invalid id goes to tile 0 in k_sp_tile_lists, which reports it)
        const bool in = p0 + 64 * k + lane < n;
        const bool valid = uint32_t(it[k]) < uint32_t(M);
        // (tile 0: a hot id after a relabel -- a bit -- else an id below kTW)
        const bool t0 = !valid || (rank_of ? bit_of(hotbm, uint32_t(it[k])) : uint32_t(it[k]) < uint32_t(kTW));
        n0 += int32_t(__popcll(__ballot(in && t0)));
        if (owner) mine += int32_t(__popcll(__ballot(valid && bit_of(minebm, uint32_t(it[k])))));
      }
    }
    if (lane == 0) {
      len[j] = (uint64_t((n0 + 7) & ~7) << 32) | uint64_t((n - n0 + 3) & ~3);
      if (owner) ownc[j] = mine;
    }
  }
}

// One wave per user: validates the ids, emits the contributions (item, user) in CSR order for the item
// sort (the keyBy(itemA) regrouping, FlinkCooccurrences.java:152; owner != NULL: only counts the owned
// ones), counts the list by tile in LDS and writes the arenas: the user's tile-0 ids as u16 at its
// arena0 base (kSink16 pads to a multiple of 8), its other ids tile by tile as u32 at its arena1 base
// (kSink pads to a multiple of 4), bases from k_sp_tile_counts' prefix.  tb[j] gets the absolute
// offsets: [0] = base0, [t] = base1 + the ids of tiles 1..t-1, [T + 1] = base0 + the tile-0 ids.
constexpr int kTlR = 4;  // ids per lane held in registers across both passes (users of <= 256 ids)

__global__ __launch_bounds__(256) void k_sp_tile_lists(int64_t U, const int64_t *__restrict__ up,
                                                       const int32_t *__restrict__ items, int32_t M, int32_t T,
                                                       int32_t *__restrict__ tb, uint16_t *__restrict__ arena0,
                                                       uint32_t *__restrict__ arena1, const uint64_t *__restrict__ pbase,
                                                       uint32_t *__restrict__ keys,
                                                       uint32_t *__restrict__ vals, const int32_t *__restrict__ owner,
                                                       int32_t part, const int64_t *__restrict__ ownoff,
                                                       PlanTotals *__restrict__ tot, const int32_t *__restrict__ rank_of,
                                                       const uint32_t *__restrict__ hotbm,
                                                       const uint32_t *__restrict__ minebm) {
  __shared__ int32_t cur[4][kSpMaxTiles + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int32_t *c = cur[wave];
  const int64_t gw = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  bool bad = false;
  int64_t s = 0, e = 0;
  if (gw < U) {
    s = up[gw];
    e = up[gw + 1];
  }
  for (int64_t j = gw; j < U; j += n_waves) {
    const int32_t n = int32_t(e - s);
    // the next user's bounds and this user's first kTlR * 64 ids: all loads in flight together
    int64_t sn = 0, en = 0;
    if (j + n_waves < U) {
      sn = up[j + n_waves];
      en = up[j + n_waves + 1];
    }
    int32_t r[kTlR];
#pragma unroll
    for (int k = 0; k < kTlR; k++) {
      const int32_t p = lane + 64 * k;
      r[k] = p < n ? items[s + p] : 0;
      if (uint32_t(r[k]) >= uint32_t(M)) bad = true;
    }
    for (int32_t t = lane; t <= T; t += 64) c[t] = 0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    int32_t n0 = 0;  // (tile-0 ids, the Zipf head, counted by ballot: no same-address LDS atomics)
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    int64_t o = owner ? ownoff[j] : 0;  // (owned contributions: at ownoff[j], in list order)
    // it: the item id (contributions, owner map); rk: its column rank (tiles, arenas)
    auto count = [&](bool in, int32_t p, int32_t it, int32_t rk, bool valid) {
      n0 += __popcll(__ballot(in && (rk >> kTShift) == 0));
      if (in && (rk >> kTShift)) atomicAdd(&c[rk >> kTShift], 1);
      if (!owner) {
        if (keys && in) {  // (NULL: the contributions come from elsewhere, k_sp_window_contribs)
          keys[s + p] = uint32_t(it);
          vals[s + p] = uint32_t(j);
        }
      } else {
        const bool m = in && valid && bit_of(minebm, uint32_t(it));
        const uint64_t bal = __ballot(m);
        if (m && keys) {
          keys[o + __popcll(bal & lt)] = uint32_t(it);
          vals[o + __popcll(bal & lt)] = uint32_t(j);
        }
        o += __popcll(bal);
      }
    };
    bool valid[kTlR];
    int32_t rk[kTlR];
#pragma unroll
    for (int k = 0; k < kTlR; k++) {
      valid[k] = uint32_t(r[k]) < uint32_t(M);
      if (!valid[k]) r[k] = 0;
      rk[k] = lane + 64 * k < n ? planner_rank(rank_of, hotbm, uint32_t(r[k])) : r[k];
    }
#pragma unroll
    for (int k = 0; k < kTlR; k++) count(lane + 64 * k < n, lane + 64 * k, r[k], rk[k], valid[k]);
    for (int32_t p0 = 64 * kTlR; p0 < n; p0 += 64) {
      const int32_t p = p0 + lane;
      int32_t it = p < n ? items[s + p] : 0;
      const bool v = uint32_t(it) < uint32_t(M);
      if (!v) {
        bad = true;
        it = 0;
      }
      count(p < n, p, it, p < n ? planner_rank(rank_of, hotbm, uint32_t(it)) : it, v);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    int32_t *tbj = tb + j * (T + 2);
    const int32_t n1 = n - n0;
    const uint64_t pb = pbase[j];
    const int64_t b0 = int64_t(pb >> 32), b1 = int64_t(pb & 0xFFFFFFFFull);
    // exclusive prefix of tiles 1..T's counts: tb and the tiles' cursors
    if (T < 64) {  // one wave scan, lane t = tile t
      const int32_t x = (lane >= 1 && lane <= T) ? c[lane] : 0;
      const int32_t ex = int32_t(wave_incl_scan(uint32_t(x))) - x;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (lane >= 1 && lane <= T) {
        tbj[lane] = int32_t(b1 + ex);  // (tile T is empty: tbj[T] = base1 + n1)
        c[lane] = ex;
      }
    } else if (lane == 0) {
      int32_t run = 0;
      for (int32_t t = 1; t <= T; t++) {
        const int32_t x = c[t];
        tbj[t] = int32_t(b1 + run);
        c[t] = run;
        run += x;
      }
    }
    if (lane == 0) {
      tbj[0] = int32_t(b0);
      tbj[T + 1] = int32_t(b0 + n0);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    uint16_t *o0 = arena0 + b0;
    uint32_t *o1 = arena1 + b1;
    int32_t q0 = 0;  // the tile-0 cursor (wave-uniform): ballot ranks, in lane order
    auto place = [&](bool in, int32_t it) {
      const bool t0 = in && (it >> kTShift) == 0;
      const uint64_t b = __ballot(t0);
      if (t0) o0[q0 + int32_t(__popcll(b & lt))] = uint16_t(it);
      else if (in) o1[atomicAdd(&c[it >> kTShift], 1)] = uint32_t(it);
      q0 += int32_t(__popcll(b));
    };
#pragma unroll
    for (int k = 0; k < kTlR; k++) place(lane + 64 * k < n, rk[k]);
    for (int32_t p0 = 64 * kTlR; p0 < n; p0 += 64) {  // (long lists: L1 / L2 lines of the first pass)
      const int32_t p = p0 + lane;
      int32_t it = p < n ? items[s + p] : 0;
      if (uint32_t(it) >= uint32_t(M)) it = 0;
      place(p < n, p < n ? planner_rank(rank_of, hotbm, uint32_t(it)) : it);
    }
    if (lane < ((n0 + 7) & ~7) - n0) o0[n0 + lane] = uint16_t(kSink16);  // (<= 7 pads)
    if (lane < ((n1 + 3) & ~3) - n1) o1[n1 + lane] = kSink;              // (<= 3 pads)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    s = sn;
    e = en;
  }
  if (bad) atomicOr(reinterpret_cast<unsigned long long *>(&tot->err), 1ull);
}

// A contribution's value: the index of the list its row walks; in a streaming window (spre != NULL) with
// kSelfBit when the walk includes the contribution's own position (a new position walks its user's whole
// history, an old one only the window's new items, see k_sp_window_contribs).  In a one-window batch every
// walk includes it (no bit: the self count of a row is its contribution count).
constexpr uint32_t kSelfBit = 0x80000000u, kListMask = 0x7FFFFFFFu;

// Streaming window (old / new positions, NonSampled...java:129-161): user j's two lists are A_j (the whole
// history after the window, at up2[2j]) and B_j (its new items, positions >= old[j], at up2[2j + 1]).
// Position p of A_j is a contribution of row x_p: a new position (p >= old[j]) walks A_j (every pair with
// it as the later one, the pair with itself removed: kSelfBit), an old one walks B_j (its pairs with the
// window's items).  Contribution p of user j lands at cbase[j] + p.  One wave per user.
__global__ __launch_bounds__(256) void k_sp_window_contribs(int64_t U, const int64_t *__restrict__ up2,
                                                           const int32_t *__restrict__ items,
                                                           const int32_t *__restrict__ old,
                                                           const int64_t *__restrict__ cbase,
                                                           uint32_t *__restrict__ keys, uint32_t *__restrict__ vals) {
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t j = gw; j < U; j += n_waves) {
    const int64_t s = up2[2 * j];
    const int32_t n = int32_t(up2[2 * j + 1] - s), o = old[j];
    const int64_t c = cbase[j];
    for (int32_t p = lane; p < n; p += 64) {
      keys[c + p] = uint32_t(items[s + p]);
      vals[c + p] = p >= o ? (uint32_t(2 * j) | kSelfBit) : uint32_t(2 * j + 1);
    }
  }
}

// The (item, user) contributions of a batch in CSR order, for the item sort (the keyBy(itemA) regrouping,
// FlinkCooccurrences.java:152) ahead of the column relabel; an invalid id (k_sp_tile_lists reports it)
// becomes row 0.  One wave per user.
__global__ __launch_bounds__(256) void k_sp_contribs(int64_t U, const int64_t *__restrict__ up,
                                                     const int32_t *__restrict__ items, int32_t M,
                                                     uint32_t *__restrict__ keys, uint32_t *__restrict__ vals) {
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t j = gw; j < U; j += n_waves) {
    const int64_t s = up[j], e = up[j + 1];
    for (int64_t p = s + lane; p < e; p += 64) {
      const int32_t it = items[p];
      keys[p] = uint32_t(it) < uint32_t(M) ? uint32_t(it) : 0u;
      vals[p] = uint32_t(j);
    }
  }
}

// Column relabel: the kTW most frequent items of the batch (its own frequencies -- the row lengths of the
// item-sorted contributions -- or the caller's global counts; ties: the smaller id first) become tile 0, in
// ascending id order; every other item keeps its id shifted one tile up.  So tile 0 (u16 arena, dense LDS
// tiles) holds the Zipf head whatever order the ids come in, and a column maps back to its item by a lookup
// in a 64 KB table (tile 0) or a subtraction (above).
__global__ void k_rank_keys(const int64_t *__restrict__ row_ptr, const int64_t *__restrict__ freq, int32_t M,
                            uint64_t *__restrict__ keys, int32_t *__restrict__ ids, uint8_t *__restrict__ hot) {
  const int32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= M) return;
  keys[a] = uint64_t(freq ? freq[a] : row_ptr[a + 1] - row_ptr[a]);
  ids[a] = a;
  hot[a] = 0;
}

__global__ void k_hot_mark(const int32_t *__restrict__ order, int32_t h, uint8_t *__restrict__ hot) {
  const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < h) hot[order[r]] = 1;
}

// how many of the hot items already have an id below kTW (the relabel is skipped when nearly all do)
__global__ void k_hot_overlap(const uint8_t *__restrict__ hot, int32_t n, int32_t *__restrict__ out) {
  const int32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c = uint32_t(__popcll(__ballot(a < n && hot[a] != 0)));
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, int32_t(c));
}

// Bitmaps over item ids for the planner's per-interaction passes: a 4-B gather per interaction into an
// M-entry table is one L2 request per lane (the passes over a whole 1e9-interaction log are bound by that
// request rate), a bit lookup into an M-bit table shares lines between the lanes (the hot ids' bits sit in
// few lines).  hot: the ids of tile 0 after a relabel; mine: the rows a part owns.
__global__ void k_bits_hot(const uint8_t *__restrict__ hot, int32_t M, uint32_t *__restrict__ bits) {
  const int32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w * 32 >= M) return;
  uint32_t v = 0;
  for (int b = 0; b < 32 && w * 32 + b < M; b++) v |= uint32_t(hot[w * 32 + b] != 0) << b;
  bits[w] = v;
}

__global__ void k_bits_owner(const int32_t *__restrict__ owner, int32_t part, int32_t M, uint32_t *__restrict__ bits) {
  const int32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w * 32 >= M) return;
  uint32_t v = 0;
  for (int b = 0; b < 32 && w * 32 + b < M; b++) v |= uint32_t(owner[w * 32 + b] == part) << b;
  bits[w] = v;
}

struct IsHot {
  const uint8_t *hot;
  __host__ __device__ bool operator()(int32_t a) const { return hot[a] != 0; }
};

// pos_of (item -> column) and the frequencies in column order (the planner's per-tile estimate; the holes of
// the hot items above tile 0 count 0)
__global__ void k_relabel_pos(const uint8_t *__restrict__ hot, const uint64_t *__restrict__ freq_by_id, int32_t M,
                              int32_t *__restrict__ pos_of, int64_t *__restrict__ freq_col) {
  const int32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= M) return;
  const bool h = hot[a] != 0;
  if (!h) pos_of[a] = a + kTW;
  freq_col[kTW + a] = h ? 0 : int64_t(freq_by_id[a]);
}

__global__ void k_relabel_hot(const int32_t *__restrict__ hot_col, const uint64_t *__restrict__ freq_by_id,
                              int32_t *__restrict__ pos_of, int64_t *__restrict__ freq_col) {
  const int32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= kTW) return;
  const int32_t a = hot_col[c];
  pos_of[a] = c;
  freq_col[c] = int64_t(freq_by_id[a]);
}


__global__ void k_sp_row_ptr(const uint32_t *__restrict__ keys, int64_t n, int32_t M, int64_t *__restrict__ row_ptr) {
  const int64_t a = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (a > M) return;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (keys[mid] < uint32_t(a)) lo = mid + 1; else hi = mid;
  }
  row_ptr[a] = lo;
}

struct UserLen {  // list length of a contribution's list
  const int64_t *up;
  __host__ __device__ int64_t operator()(uint32_t u) const { return up[(u & kListMask) + 1] - up[u & kListMask]; }
};

struct ScanUserLen {  // the pair work of contribution i (its list's length, from the u32 table), for launch_scan
  const uint32_t *vals;
  const uint32_t *len;
  __device__ int64_t operator()(int64_t i) const { return int64_t(len[vals[i] & kListMask]); }
};

// the lists' lengths as u32 (one 4-B gather per contribution in the pair-work prefix instead of two 8-B ones
// from the CSR pointers: a 5-MB table at the 1/8 C3 share)
__global__ void k_list_len32(int64_t U, const int64_t *__restrict__ up, uint32_t *__restrict__ len) {
  const int64_t u = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (u < U) len[u] = uint32_t(up[u + 1] - up[u]);
}

struct SelfFlag {  // 1 for a contribution whose walk includes its own position
  __host__ __device__ int64_t operator()(uint32_t u) const { return int64_t(u >> 31); }
};
struct ScanSelfFlag {  // SelfFlag of contribution i, for launch_scan
  const uint32_t *vals;
  __device__ int64_t operator()(int64_t i) const { return int64_t(vals[i] >> 31); }
};

// est[t][k] = sum over the columns b of tile t of 1 - exp(-2^(k/2) f_b / N); gmass[t] = tile t's
// share of the interactions.  One block per (tile, k).
__global__ __launch_bounds__(256) void k_sp_est(const int64_t *__restrict__ row_ptr, const int64_t *__restrict__ freq,
                                                int32_t M, int64_t n, float *__restrict__ est, float *__restrict__ gmass) {
  __shared__ double s_mass[4];
  __shared__ float s[4];
  const int t = blockIdx.x, k = blockIdx.y;
  const int32_t b0 = t * kTW, b1 = min(M, b0 + kTW);
  const float scale = exp2f(0.5f * float(k)) / float(n);
  float acc = 0.f;
  double mass = 0.0;
  for (int32_t b = b0 + threadIdx.x; b < b1; b += 256) {
    const int64_t fi = freq ? freq[b] : row_ptr[b + 1] - row_ptr[b];
    const float f = float(fi);
    mass += double(fi);
    if (f > 0.f) acc += -expm1f(-f * scale);
  }
  for (int o = 32; o > 0; o >>= 1) {
    acc += __shfl_xor(acc, o, 64);
    mass += __shfl_xor(mass, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    s[threadIdx.x >> 6] = acc;
    s_mass[threadIdx.x >> 6] = mass;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    est[t * kEstK + k] = s[0] + s[1] + s[2] + s[3];
    if (k == 0) gmass[t] = float((s_mass[0] + s_mass[1] + s_mass[2] + s_mass[3]) / double(n));
  }
}

// Per row: pair work W_a (exact), row sum W_a - c_a (closed form), and the chunk plan.
__global__ __launch_bounds__(256) void k_sp_plan(int32_t M, int32_t T, const int64_t *__restrict__ row_ptr,
                                                 const int64_t *__restrict__ epre, const float *__restrict__ est,
                                                 const float *__restrict__ gmass, int64_t *__restrict__ rowsum,
                                                 int64_t *__restrict__ row_w, uint64_t *__restrict__ pstart,
                                                 uint64_t *__restrict__ pdense, uint64_t *__restrict__ hz,
                                                 uint64_t *__restrict__ skey,
                                                 int32_t *__restrict__ order, int32_t *__restrict__ nwork,
                                                 int32_t *__restrict__ row_nnz, int64_t *__restrict__ row_base,
                                                 PlanTotals *__restrict__ tot, const int64_t *__restrict__ spre,
                                                 int32_t tiny_on) {
  __shared__ uint64_t s_red[4][4];
  const int32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t est_sum = 0, bound = 0, n_split = 0, split_work = 0, n_active = 0, max_tail = 0, n_gather = 0, n_tiny = 0,
           n_small = 0, ts_pairs = 0, n_mid = 0, max_tail_mid = 0;
  if (a < M) {
    const int64_t k0 = row_ptr[a], c = row_ptr[a + 1] - k0;
    const int64_t W = epre[k0 + c] - epre[k0];
    const int64_t self = spre ? spre[k0 + c] - spre[k0] : c;  // pairs of a position with itself
    rowsum[a] = W - self;
    row_w[a] = W;
    row_nnz[a] = 0;
    row_base[a] = 0;
    order[a] = a;
    skey[a] = uint64_t(W);
    uint64_t st = 0, dn = 0, h0 = 0, h1 = 0;
    int32_t nw = 0;
    if (c > 0) {
      n_active = 1;
      n_tiny = ((tiny_on & 1) && W <= kTinyW) ? 1 : 0;  // (the W-descending queue puts them last)
      n_small = ((tiny_on & 2) && W > kTinyW && W <= kSmallW) ? 1 : 0;  // (... just before the tiny ones)
      ts_pairs = (n_tiny || n_small) ? uint64_t(W) : 0u;
      // a mid row (k_sp_main's 256-thread shape): its chunks are planned for 4K-slot tables over <= 2^19 columns
      const bool mid = (tiny_on & 4) && !n_tiny && !n_small && W <= kMidW;
      n_mid = mid ? 1 : 0;
      const float hfill = mid ? kHashFillMid : kHashFill, dkeys = mid ? kDenseKeysMid : kDenseKeys;
      const int hmax = mid ? SpMid::kHashMax : kHashMax;
      const int hmaxtiles = mid ? SpMid::kHashMaxTiles : kHashMaxTiles;
      bound = uint64_t(min<int64_t>(W - self, M));
      float e_tot = 0.f;
      if (W > kSplitWork) {
        n_split = 1;
        for (int t = 0; t < T; t++) e_tot += est_distinct(est, t, W);
        nw = sp_split_shares(W, gmass[0]);
        split_work = uint64_t(nw);
        max_tail = uint64_t(float(W) * fmaxf(0.f, 1.f - gmass[0]) / float(nw));
      } else {
        float cur = 0.f;
        int n_in = 0, cs = -1;
        // a hash chunk's table: the smallest power of two >= SLACK * E[distinct] + 64 slots (kHashMin..kHashMax)
        auto close = [&]() {
          if (cs < 0) return;
          uint64_t code = 0;
#ifndef COOC_SP_HASH_SLACK
#define COOC_SP_HASH_SLACK 4.f  // table >= 4x the estimated distinct count (A/B)
#endif
          for (int H = kHashMin; H < hmax && float(H) < COOC_SP_HASH_SLACK * cur + 64.f; H <<= 1) code++;
          if (cs < 32) h0 |= code << (2 * cs); else h1 |= code << (2 * (cs - 32));
          cs = -1;
        };
        for (int t = 0; t < T; t++) {
          const float d = est_distinct(est, t, W);
          const float e = float(W) * gmass[t];
          e_tot += d;
          if (d > dkeys || e > kDensePairs) {
            close();
            st |= uint64_t(1) << t;
            dn |= uint64_t(1) << t;
          } else {
            if (cs < 0 || cur + d > hfill || n_in == hmaxtiles) {
              close();
              st |= uint64_t(1) << t;
              cs = t;
              cur = 0.f;
              n_in = 0;
            }
            cur += d;
            n_in++;
          }
        }
        close();
        if ((dn & 1ull) && __popcll(st) >= kGatherMinChunks) {  // gather mode (k_sp_main)
          // the flag: bit 0 of tile 0's hash-size code, unused when tile 0 is dense (every bit of dn is a
          // tile: a 64-tile universe, 1,032,193 to 1,048,576 columns, has one in bit 63)
          h0 |= kGatherFlag;
          max_tail = uint64_t(float(W) * fmaxf(0.f, 1.f - gmass[0]));
          if (mid) {
            max_tail_mid = max_tail;
            max_tail = 0;
          }
          n_gather = 1;
        }
      }
      est_sum = uint64_t(e_tot) + 1;
      row_nnz[a] = int32_t(min(est_sum, uint64_t(INT32_MAX)));  // carried to the queue record (k_sp_queue)
    }
    pstart[a] = st;
    pdense[a] = dn;
    hz[2 * a] = h0;
    hz[2 * a + 1] = h1;
    nwork[a] = nw;
  }
  uint64_t v[4] = {est_sum, bound, n_split, split_work};
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = 0; i < 4; i++) {
    for (int o = 32; o > 0; o >>= 1) v[i] += __shfl_xor(v[i], o, 64);
    if (lane == 0) s_red[i][w] = v[i];
  }
  uint64_t act = n_active;
  for (int o = 32; o > 0; o >>= 1) {
    act += __shfl_xor(act, o, 64);
    n_tiny += __shfl_xor(n_tiny, o, 64);
    n_small += __shfl_xor(n_small, o, 64);
    n_mid += __shfl_xor(n_mid, o, 64);
    max_tail_mid = max(max_tail_mid, __shfl_xor(max_tail_mid, o, 64));
    ts_pairs += __shfl_xor(ts_pairs, o, 64);
    n_gather += __shfl_xor(n_gather, o, 64);
    max_tail = max(max_tail, __shfl_xor(max_tail, o, 64));
  }
  if (lane == 0 && max_tail) atomicMax(reinterpret_cast<unsigned long long *>(&tot->max_tail), (unsigned long long)max_tail);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t r[4];
    for (int i = 0; i < 4; i++) r[i] = s_red[i][0] + s_red[i][1] + s_red[i][2] + s_red[i][3];
    if (r[0]) atomicAdd(reinterpret_cast<unsigned long long *>(&tot->est_nnz), (unsigned long long)r[0]);
    if (r[1]) atomicAdd(reinterpret_cast<unsigned long long *>(&tot->cap_total), (unsigned long long)r[1]);
    if (r[2]) atomicAdd(reinterpret_cast<unsigned long long *>(&tot->n_split), (unsigned long long)r[2]);
    if (r[3]) atomicAdd(reinterpret_cast<unsigned long long *>(&tot->n_split_work), (unsigned long long)r[3]);
  }
  if (lane == 0 && act) atomicAdd(reinterpret_cast<unsigned long long *>(&tot->n_active), (unsigned long long)act);
  if (lane == 0 && n_tiny) atomicAdd(reinterpret_cast<unsigned long long *>(&tot->n_tiny), (unsigned long long)n_tiny);
  if (lane == 0 && n_small) atomicAdd(reinterpret_cast<unsigned long long *>(&tot->n_small), (unsigned long long)n_small);
  if (lane == 0 && n_mid) atomicAdd(reinterpret_cast<unsigned long long *>(&tot->n_mid), (unsigned long long)n_mid);
  if (lane == 0 && max_tail_mid)
    atomicMax(reinterpret_cast<unsigned long long *>(&tot->max_tail_mid), (unsigned long long)max_tail_mid);
  if (lane == 0 && ts_pairs) atomicAdd(reinterpret_cast<unsigned long long *>(&tot->ts_pairs), (unsigned long long)ts_pairs);
  if (lane == 0 && n_gather)
    atomicAdd(reinterpret_cast<unsigned long long *>(&tot->n_gather_rows), (unsigned long long)n_gather);
}

__global__ void k_sp_gather_nwork(const int32_t *__restrict__ order, const int32_t *__restrict__ nwork, int32_t M,
                                  int32_t *__restrict__ out) {
  const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < M) out[r] = nwork[order[r]];
}

// Work queue: the split rows' shares (they are the heaviest rows, so the first n_split rows of the
// W-descending order), then every other row with contributions, heaviest first.  Gather items get a
// row of bucket starts (gslot).
__global__ void k_sp_queue(const int32_t *__restrict__ order, const uint64_t *__restrict__ skey,
                           const int32_t *__restrict__ wbase, const float *__restrict__ gmass,
                           const int64_t *__restrict__ row_ptr, const uint64_t *__restrict__ pstart,
                           const uint64_t *__restrict__ pdense, const uint64_t *__restrict__ hz, int32_t M, int32_t T,
                           PlanTotals *__restrict__ tot, SpWork *__restrict__ queue, int32_t *__restrict__ split_slot,
                           int32_t *__restrict__ split_row, const int32_t *__restrict__ row_nnz) {
  const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= M) return;
  const int64_t n_split = tot->n_split, n_split_work = tot->n_split_work;
  const int32_t a = order[r];
  const int64_t W = int64_t(skey[r]);
  if (W <= 0) return;
  const int64_t r0 = row_ptr[a], r1 = row_ptr[a + 1];
  unsigned long long *ng = reinterpret_cast<unsigned long long *>(&tot->n_gather);
  if (r < n_split) {
    split_slot[a] = r;
    split_row[r] = a;
    const int64_t q = wbase[r];
    const int32_t ns = sp_split_shares(W, gmass[0]);
    for (int32_t s = 0; s < ns; s++) {
      SpWork x{};
      x.k0 = r0 + (r1 - r0) * s / ns;
      x.k1 = r0 + (r1 - r0) * (s + 1) / ns;
      x.row = a;
      x.kind = -2;
      x.gslot = int32_t(atomicAdd(ng, 1ull));
      queue[q + s] = x;
    }
  } else {
    SpWork x{};
    x.k0 = r0;
    x.k1 = r1;
    x.st = pstart[a];
    x.dn = pdense[a];
    x.hz[0] = hz[2 * a];
    x.hz[1] = hz[2 * a + 1];
    x.row = a;
    x.kind = -1;
    x.gslot = ((x.dn & 1ull) && (x.hz[0] & kGatherFlag)) ? int32_t(atomicAdd(ng, 1ull)) : -1;
    x.est = row_nnz[a];
    queue[n_split_work + (r - n_split)] = x;
  }
}

__global__ void k_sp_totals(PlanTotals *__restrict__ tot, const int64_t *__restrict__ epre,
                            const int64_t *__restrict__ spre, int64_t n, int32_t *__restrict__ qctr) {
  tot->n_chunks = tot->n_split_work + (tot->n_active - tot->n_split);
  tot->work_total = epre[n];
  tot->self_total = spre ? spre[n] : n;
  qctr[0] = qctr[1] = 0;
}

// ---- the accumulate kernel --------------------------------------------------------------------------
struct SpShared {
  uint32_t *R;       // [kTW] dense counters | hash keys [0, H) + counts [kHashMax, kHashMax + H)
  uint32_t *L1;      // [kL1Words] hash compaction: one bit per 32-column block
  uint32_t *L1pre;   // [kL1Words] its exclusive popcount prefix
  int32_t *gb;       // [kSpDb] a segment's first 16-B group - its virtual start
  uint32_t *info;    // [kSpDb] (its end - its first group's first position) << 2 | its first id's lane
  uint32_t *vst;     // [kSpDb + 1] virtual starts
  int32_t *qstart;   // [256] first segment of every walker
};

struct SpStatic {
  uint32_t wtot[kSpWaves];
  uint64_t red[kSpWaves];
  int32_t work;
  uint32_t flag;
  int64_t slab_cur, slab_end, row_begin, row_n, pos, copy_from, copy_n;
  int64_t saved_cur, saved_end;  // the workgroup's slab while a big row fills a region of its own
  uint32_t own;
  uint32_t bstart[kSpMaxTiles + 1]; // gather mode: bucket starts in the workgroup's scratch
  uint32_t bcur[kSpMaxTiles];       // ... and fill cursors
  uint64_t ovf;                     // tiles whose bucket overflowed (their chunks walk the lists)
  unsigned long long rsum;          // the current whole row's compacted counts, summed (row-sum check)
#ifdef COOC_SP_STATS
  unsigned long long st[64];
#endif
};

// Insert the (up to 4) partner ids of one 16-B group into the LDS table (keys store id + 1; 0 =
// empty), linear probing from a multiplicative hash.  The ids are probed in lockstep so that their
// LDS round trips overlap; each probe is one returning compare-and-swap (it claims an empty slot or
// returns the key that holds it) followed, on a hit, by a non-returning count add.  An id that finds
// no slot within kMaxProbe probes raises the overflow flag (the chunk is redone with a larger table);
// the planner sizes tables at <= 1/2 fill, so probe chains stay short.
__device__ inline void sp_hash_insert4(uint32_t *keys, uint32_t *cnts, const uint4 &v, uint32_t hshift, uint32_t hmask,
                                       SpStatic &S_) {
  uint32_t k[4] = {v.x + 1u, v.y + 1u, v.z + 1u, v.w + 1u};  // kSink + 1 == 0: a pad is never inserted
  uint32_t h[4];
#pragma unroll
  for (int i = 0; i < 4; i++) h[i] = (k[i] - 1u) * 0x9E3779B1u >> hshift;
#ifdef COOC_SP_STATS
  if (threadIdx.x == 0) S_.st[24] += (k[0] != 0u) + (k[1] != 0u) + (k[2] != 0u) + (k[3] != 0u);
#endif
  for (int p = 0; p < kMaxProbe; p++) {
#ifdef COOC_SP_STATS
    if (threadIdx.x == 0) S_.st[25] += 1;
#endif
    uint32_t cur[4];
#pragma unroll
    for (int i = 0; i < 4; i++) cur[i] = k[i] ? atomicCAS(keys + h[i], 0u, k[i]) : 0u;
    bool left = false;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if (!k[i]) continue;
      if (cur[i] == 0u || cur[i] == k[i]) {
        atomicAdd(cnts + h[i], 1u);
        k[i] = 0u;
      } else {
        h[i] = (h[i] + 1u) & hmask;
        left = true;
      }
    }
    if (!left) return;
  }
  S_.flag = 1u;
}

struct WalkOp {
  int mode;  // 0: dense counters R[id - c0]; 1: hash insert; 2: gather (tile 0 dense, other tiles to buckets)
  uint32_t c0, hshift, hmask;
  int64_t sbase;  // gather: the workgroup's scratch (16-B groups)
};

// One 16-B group of kIds partner ids (kIds = 4: u32 ids of arena1 or a gather bucket; 8: u16 tile-0 ids
// of arena0); m = the lanes (bits 0 .. kIds - 1) inside the walked segment, the others are ids of a
// neighbouring tile range or list (or end-of-list sinks) and are skipped.  Gather mode: an id of tile 0
// is counted in the dense tile, any other is appended to its tile's bucket (4-B ids, packed).
// A +1 at dense counter o of the LDS tile: u32 counters, or (mid shape) u16 counters packed two per word.
template <class Sh>
__device__ inline void sp_dense_add(uint32_t *R, uint32_t o) {
  if (Sh::kU16)
    atomicAdd(&R[o >> 1], 1u << ((o & 1u) << 4));
  else
    atomicAdd(&R[o], 1u);
}

template <class Sh, int kIds>
__device__ inline void sp_apply_group(const SpArgs &A, const SpShared &L, SpStatic &S_, const WalkOp &op,
                                      const uint4 &v, uint32_t m) {
  uint32_t x[kIds];
  if (kIds == 4) {
    x[0] = v.x;
    x[1] = v.y;
    x[2] = v.z;
    x[3] = v.w;
  } else {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
      x[2 * i] = w[i] & 0xFFFFu;
      x[2 * i + 1] = w[i] >> 16;
    }
  }
#pragma unroll
  for (int i = 0; i < kIds; i++)
    if (!((m >> i) & 1u)) x[i] = kSink;
#ifdef COOC_SP_STATS
  if (A.exp == 1 && op.mode == 1) {  // timing experiment: hash chunks load their groups but insert nothing
    if (x[1] == 0xFFFFFFFEu) S_.flag = 1u;
    return;
  }
#endif
  if (op.mode == 1) {
#pragma unroll
    for (int h = 0; h < kIds; h += 4)
      sp_hash_insert4(L.R, L.R + Sh::kHashMax, make_uint4(x[h], x[h + 1], x[h + 2], x[h + 3]), op.hshift, op.hmask, S_);
    return;
  }
  if (op.mode == 2) {
    uint32_t *scr = reinterpret_cast<uint32_t *>(A.scratch + op.sbase);
#pragma unroll
    for (int i = 0; i < kIds; i++) {
      if (x[i] == kSink) continue;
      const uint32_t t = x[i] >> kTShift;
      if (t == 0) {
        sp_dense_add<Sh>(L.R, x[i]);
      } else {
        const uint32_t slot = atomicAdd(&S_.bcur[t], 1u);
        if (slot < S_.bstart[t + 1] - S_.bstart[t]) scr[S_.bstart[t] + slot] = x[i];  // else the bucket overflowed
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < kIds; i++)
    if (x[i] != kSink) sp_dense_add<Sh>(L.R, x[i] - op.c0);
}

// One batch of segments: this thread's segment (tid < nb) is the ids at positions [s, e) of ar (16-B
// groups of kIds ids; a segment starts and ends anywhere inside a group).  The segments' group counts
// are block-scanned into virtual starts; walkers of S lanes (S from the mean segment length) own equal
// contiguous shares of the virtual range and step S groups at a time, kSpU loads in flight per lane,
// applying op to every id of the segment (lanes outside it masked).  Returns the batch's groups
// (uniform); ends with a barrier.
template <class Sh, int kIds>
__device__ inline uint32_t sp_walk_batch(const SpArgs &A, const SpShared &L, SpStatic &S_, const uint4 *__restrict__ ar,
                                         int64_t nsrc, int nb, uint32_t s, uint32_t e, const WalkOp &op) {
  constexpr uint32_t kSh = kIds == 8 ? 3u : 2u, kLo = kIds - 1;
  const int tid = threadIdx.x;
  const unsigned long long c_b0 = STAT_CLOCK();
  const uint32_t len = (tid < nb && e > s) ? ((e + kLo) >> kSh) - (s >> kSh) : 0u;
  uint32_t total;
  const uint32_t ex = block_excl_scan<Sh::kWaves>(len, &total, S_.wtot);
  if (total == 0) return 0;  // uniform (scalar branch): no barrier is skipped by part of the block
  const uint32_t mean = total / uint32_t(nb);
#ifndef COOC_SP_SLONG
#define COOC_SP_SLONG 64u  // whole-wave walkers for long segments: 1.2% faster than 16 (profiles/r03/walker_ab)
#endif
#ifndef COOC_SP_SSHORT
#define COOC_SP_SSHORT 4u
#endif
#ifndef COOC_SP_STIER
#define COOC_SP_STIER 32  // segments of >= 32 groups: whole-wave walkers, >= 12: 16 lanes (profiles/r03/walker_ab)
#endif
  const uint32_t S = mean >= COOC_SP_STIER ? COOC_SP_SLONG : mean >= 12 ? 16u : COOC_SP_SSHORT;
  const uint32_t nW = uint32_t(Sh::kThreads) / S;
  if (tid < nb) {
    L.vst[tid] = ex;
    L.gb[tid] = int32_t(s >> kSh) - int32_t(ex);
    L.info[tid] = ((e - (s & ~kLo)) << 3) | (s & kLo);
    if (len) {
      const uint32_t q0 = uint32_t((uint64_t(ex) * nW + total - 1) / total);
      const uint32_t q1 = uint32_t((uint64_t(ex + len) * nW + total - 1) / total);
      for (uint32_t q = q0; q < q1 && q < nW; q++) L.qstart[q] = tid;
    }
  }
  if (tid == 0) L.vst[nb] = total;
  __syncthreads();
  const unsigned long long c_b1 = STAT_CLOCK();
  if (op.mode == 1) STAT_ADD(16, c_b1 - c_b0);
  if (op.mode == 1) STAT_ADD(18, total);
  const uint32_t q = uint32_t(tid) / S, ql = uint32_t(tid) % S;
  const uint32_t lo = uint32_t(uint64_t(total) * q / nW), hi = uint32_t(uint64_t(total) * (q + 1) / nW);
  uint32_t g = lo + ql;
  if (g < hi) {
    int32_t cur = L.qstart[q];
    uint32_t vs = L.vst[cur], next = L.vst[cur + 1], inf = L.info[cur];
    int32_t gb = L.gb[cur];
    // the group at virtual index gk of the current segment, and its in-segment lanes
    auto fetch = [&](uint32_t gk, uint4 &v, uint32_t &m) {
      while (gk >= next) {
        cur++;
        vs = next;
        next = L.vst[cur + 1];
        gb = L.gb[cur];
        inf = L.info[cur];
      }
      int64_t gi = int64_t(gb) + int64_t(gk);
#ifdef COOC_SP_STATS
      if (A.exp == 2 && op.mode != 2 && (gk & 1u)) gi = -1;  // (the experiment below: no load)
#endif
      const uint32_t qq = gk - vs;
      const uint32_t lo_l = qq ? 0u : (inf & 7u);
      const int32_t hi_l = min(int32_t(kIds), int32_t(inf >> 3) - int32_t(kIds) * int32_t(qq));
      m = ((1u << hi_l) - 1u) & ~((1u << lo_l) - 1u);
#ifdef COOC_SP_STATS
      if (gi < 0) {
        v = make_uint4(kSink, kSink, kSink, kSink);
        m = 0;
        return;
      }
#endif
      v = BCHK(A, gi >= 0 && gi < nsrc, 8) ? ar[gi] : make_uint4(kSink, kSink, kSink, kSink);
    };
    uint4 v[kSpU] = {};
    uint32_t m = 0;  // 8 lane bits per group in flight
#ifdef COOC_SP_STATS
    const unsigned long long c_issue = STAT_CLOCK();
    bool first_seen = false;
#endif
#pragma unroll
    for (int k = 0; k < kSpU; k++) {
      const uint32_t gk = g + S * k;
      uint32_t mk = 0;
      if (gk < hi) fetch(gk, v[k], mk);
      m |= mk << (8 * k);
    }
    for (; g < hi; g += S * kSpU) {
      uint4 vn[kSpU] = {};
      uint32_t mn = 0;
#pragma unroll
      for (int k = 0; k < kSpU; k++) {
        const uint32_t gk = g + S * (kSpU + k);
        uint32_t mk = 0;
        if (gk < hi) fetch(gk, vn[k], mk);
        mn |= mk << (8 * k);
      }
#pragma unroll
      for (int k = 0; k < kSpU; k++) {
        // (stats build, COOC_SP_EXP=2, results invalid: every other group of dense / hash walks is neither
        // loaded nor applied -- how much of a walk is the group delivery)
        const uint32_t mk = (m >> (8 * k)) & 255u;
        if (mk) sp_apply_group<Sh, kIds>(A, L, S_, op, v[k], mk);
#ifdef COOC_SP_STATS
        if (op.mode == 1 && k == 0 && !first_seen) {  // thread 0: the first group's data arrived and was applied
          first_seen = true;
          if (threadIdx.x == 0) {
            S_.st[54] += STAT_CLOCK() - c_issue;
            S_.st[55] += 1;
          }
        }
#endif
      }
#pragma unroll
      for (int k = 0; k < kSpU; k++) v[k] = vn[k];
      m = mn;
    }
  }
  __syncthreads();
  if (op.mode == 1) STAT_ADD(17, STAT_CLOCK() - c_b1);
  return total;
}

// Walk the partner ids of contributions [k0, k1) restricted to tiles [t0, t1) (full: whole lists),
// applying op to every id: the tile-0 part of the lists from arena0 (u16, 8 ids per load), the rest from
// arena1 (u32), a batch of kSpDb contributions at a time.  Returns the groups walked.
template <class Sh>
__device__ inline uint64_t sp_walk(const SpArgs &A, const SpShared &L, SpStatic &S_, int64_t k0, int64_t k1, int t0,
                                   int t1, bool full, const WalkOp &op) {
  uint64_t walked = 0;
  const int tid = threadIdx.x;
  const bool okt = BCHK(A, t0 >= 0 && t1 <= A.T && t0 <= t1, 4);
  const bool has0 = full || t0 == 0;                 // (uniform)
  const int ta = full ? 1 : max(t0, 1), tz = full ? A.T : t1;
  const bool has1 = tz > ta;
  for (int64_t b0 = k0; b0 < k1; b0 += Sh::kDb) {
    const int nb = int(min<int64_t>(Sh::kDb, k1 - b0));
    uint32_t s0 = 0, e0 = 0, s1 = 0, e1 = 0;
    STAT_ADD(19, op.mode == 1 ? 1 : 0);
    if (tid < nb && okt) {
      const uint32_t u = BCHK(A, b0 + tid < A.n_contrib, 1) ? A.vals[b0 + tid] & kListMask : 0u;
      const int32_t *tbu = A.tb + int64_t(BCHK(A, u < A.n_users, 2) ? u : 0u) * (A.T + 2);
      if (has0) {
        s0 = uint32_t(tbu[0]);
        e0 = uint32_t(tbu[A.T + 1]);
      }
      if (has1) {
        s1 = uint32_t(tbu[ta]);
        e1 = uint32_t(tbu[tz]);
      }
    }
    if (has0) walked += sp_walk_batch<Sh, 8>(A, L, S_, A.tarena0, A.n_groups0, nb, s0, e0, op);
    if (has1) walked += sp_walk_batch<Sh, 4>(A, L, S_, A.tarena, A.n_groups, nb, s1, e1, op);
    if (uni(S_.flag)) break;
  }
  return walked;
}

// Global stores of this workgroup made visible to its own later global loads.  __syncthreads() only
// drains LDS traffic (s_waitcnt lgkmcnt(0)), and the CU's vector L1 is write-through without
// keeping its lines in step with later stores: a line loaded earlier -- by this workgroup, or by the
// other workgroup resident on the CU reading its own data next to ours -- can still hold what the
// line had before.  So every wave waits for all its memory operations (s_waitcnt 0), the barrier,
// then the L1 is invalidated (agent-scope acquire: buffer_inv sc1) and the loads that follow read
// the XCD's L2, where the stores are.  Used where the kernel reads back what it wrote: a row moving
// to a new slab, the gather buckets.
__device__ inline void sp_global_sync() {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// Output space for n more entries of the current row (thread-uniform call).  Moves the row's
// entries so far to a new slab when the workgroup's slab is exhausted.  Returns the write position
// (-1 when the output region is exhausted: the host reruns with a larger region).
template <class Sh>
__device__ inline int64_t sp_reserve(const SpArgs &A, SpStatic &S_, int64_t n) {
  const int tid = threadIdx.x;
  if (tid == 0) {
    S_.copy_n = 0;
    if (S_.slab_cur + n > S_.slab_end) {
      const int64_t need = S_.row_n + n;
      const int64_t take = max(A.slab, need + need / 2);  // a growing row moves O(log) times
      int64_t b = int64_t(atomicAdd(A.bump, (unsigned long long)take));
      if (b + take > A.cap) {
        atomicOr(reinterpret_cast<unsigned long long *>(&A.tot->err), 4ull);
        S_.pos = -1;
      } else {
        S_.copy_from = S_.row_begin;
        S_.copy_n = S_.row_n;
        S_.row_begin = b;
        S_.slab_cur = b + S_.row_n;
        S_.slab_end = b + take;
        S_.pos = S_.slab_cur;
        S_.slab_cur += n;
      }
    } else {
      S_.pos = S_.slab_cur;
      S_.slab_cur += n;
    }
    if (S_.pos >= 0) S_.row_n += n;
  }
  __syncthreads();
  const int64_t cn = uni(S_.copy_n);
  if (cn > 0) {  // the row's earlier entries follow it to the new slab (rare)
    sp_global_sync();  // they were just stored by other waves
    const int64_t from = S_.copy_from, to = S_.row_begin;
    for (int64_t i = tid; i < cn; i += Sh::kThreads) {
      if (BCHK(A, to + i < A.cap && from + i < A.cap && from >= 0, 32)) {
        A.col_out[to + i] = A.col_out[from + i];
        A.cnt_out[to + i] = A.cnt_out[from + i];
      }
    }
  }
  return uni(S_.pos);
}

// Column-order compaction of w dense counters (16-B aligned), appended to the row's output; the
// counters are left zero.  Waves own (64 kPer)-column-aligned ranges, kPer counters per lane (one 16-B LDS
// read: 4 u32 counters, or 8 u16 ones in the mid shape).
template <class Sh>
__device__ inline void sp_dense_compact(const SpArgs &A, const SpShared &L, SpStatic &S_, int32_t w, int32_t c0,
                                        uint64_t &rsum) {
  constexpr int kPer = Sh::kPer, kStep = 64 * kPer, kQ = kPer / 4;  // kQ: 16-B id loads per lane and step
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned long long c_d0 = STAT_CLOCK();
  uint32_t *row = L.R;
  const int32_t per = ((w + Sh::kWaves - 1) / Sh::kWaves + kStep - 1) & ~(kStep - 1);
  const int32_t lo = min(w, wave * per), hi = min(w, lo + per);
  const uint4 *row4 = reinterpret_cast<const uint4 *>(row);
  auto load = [&](int32_t b, uint32_t v[kPer]) {  // counters b .. b + kPer - 1 (b a multiple of kPer)
    if (b < hi) {
      const uint4 q = row4[b / kPer];
      const uint32_t ww[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < kPer; k++) {
        const uint32_t x = Sh::kU16 ? (ww[k >> 1] >> (16 * (k & 1))) & 0xFFFFu : ww[k & 3];
        v[k] = b + k < hi ? x : 0u;
      }
    } else {
#pragma unroll
      for (int k = 0; k < kPer; k++) v[k] = 0u;
    }
  };
  uint32_t cnt = 0;
  for (int32_t b0 = lo; b0 < hi; b0 += kStep) {
    uint32_t v[kPer];
    load(b0 + kPer * lane, v);
#pragma unroll
    for (int k = 0; k < kPer; k++) cnt += v[k] != 0u;
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if (lane == 0) S_.wtot[wave] = cnt;
  __syncthreads();
  STAT_ADD(48, STAT_CLOCK() - c_d0);
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int wv = 0; wv < Sh::kWaves; wv++) {
    const uint32_t x = S_.wtot[wv];
    off += wv < wave ? x : 0u;
    tot += x;
  }
  // after a relabel the output ids of tile 0 are hot_col[b]: 16-B loads of the lane's kPer ids, two steps
  // ahead (their latency overlaps the reservation and the steps before); above tile 0 they are c0 + b - kTW
  const bool map = A.hot_col != nullptr && c0 == 0;
  auto colq = [&](int32_t b, uint4 q[kQ]) {
#pragma unroll
    for (int j = 0; j < kQ; j++)
      q[j] = (map && b < hi) ? *reinterpret_cast<const uint4 *>(A.hot_col + b + 4 * j) : make_uint4(0u, 0u, 0u, 0u);
  };
  uint4 q0[kQ], q1[kQ];
  colq(lo + kPer * lane, q0);
  colq(lo + kStep + kPer * lane, q1);
  const int64_t base = sp_reserve<Sh>(A, S_, tot);  // (barrier: every wave has read wtot)
  STAT_ADD(49, STAT_CLOCK() - c_d0);
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int32_t b0 = lo; b0 < hi; b0 += kStep) {
    const int32_t b = b0 + kPer * lane;
    uint32_t ids[kPer];
#pragma unroll
    for (int j = 0; j < kQ; j++) {
      ids[4 * j] = q0[j].x;
      ids[4 * j + 1] = q0[j].y;
      ids[4 * j + 2] = q0[j].z;
      ids[4 * j + 3] = q0[j].w;
      q0[j] = q1[j];
    }
    colq(b0 + 2 * kStep + kPer * lane, q1);
    uint32_t v[kPer];
    load(b, v);
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < kPer; k++) c += v[k] != 0u;
    const uint64_t m0 = __ballot(c & 1u), m1 = __ballot(c & 2u), m2 = __ballot(c & 4u);
    const uint64_t m3 = kPer > 4 ? __ballot(c & 8u) : 0ull;
    const uint32_t pre = uint32_t(__popcll(m0 & lt_mask)) + 2u * uint32_t(__popcll(m1 & lt_mask)) +
                         4u * uint32_t(__popcll(m2 & lt_mask)) + 8u * uint32_t(__popcll(m3 & lt_mask));
#pragma unroll
    for (int k = 0; k < kPer; k++) rsum += v[k];
    if (c) {
      int64_t pos = base + off + pre;
#pragma unroll
      for (int k = 0; k < kPer; k++) {
        if (!v[k]) continue;
        if (base >= 0) {
          if (BCHK(A, pos >= 0 && pos < A.cap, 64)) {
            A.col_out[pos] = map ? int32_t(ids[k]) : c0 + b + k - (A.hot_col ? kTW : 0);
            A.cnt_out[pos] = v[k];
          }
        }
        pos++;
      }
      // (counters past hi are never incremented -- no id reaches them -- so the whole 16-B word is cleared)
      reinterpret_cast<uint4 *>(row)[b / kPer] = make_uint4(0u, 0u, 0u, 0u);
    }
    off += uint32_t(__popcll(m0)) + 2u * uint32_t(__popcll(m1)) + 4u * uint32_t(__popcll(m2)) +
           8u * uint32_t(__popcll(m3));
  }
  STAT_ADD(50, STAT_CLOCK() - c_d0);
  __syncthreads();
  STAT_ADD(51, STAT_CLOCK() - c_d0);
}

// Column-order compaction of the hash table (H slots) of the column range [c0, c1), appended to the
// row's output; leaves the table, L1 and the scratch it uses zero.  Entries are kept in registers
// (H / kThreads <= 16 per thread); their 32-column blocks are ranked through the L1 bitmap, every
// block gets a 32-bit column mask (in the keys area) and a base (prefix of mask popcounts, in the
// counts area); an entry goes to base + popcount(mask below its column).
template <class Sh>
__device__ inline void sp_hash_compact(const SpArgs &A, const SpShared &L, SpStatic &S_, int32_t H, int32_t c0,
                                       int32_t c1, uint64_t &rsum) {
  const int tid = threadIdx.x;
  const unsigned long long c_h0 = STAT_CLOCK();
  uint32_t *keys = L.R, *cnts = L.R + Sh::kHashMax;
  const int per = H / Sh::kThreads;
  const int32_t nL1 = (c1 - c0 + 1023) >> 10;
  uint32_t ek[Sh::kHashMax / Sh::kThreads], ec[Sh::kHashMax / Sh::kThreads], er[Sh::kHashMax / Sh::kThreads];
  // the table swept 4 slots (16 B) per LDS access: thread tid takes slots 4 (tid + q kThreads) .. + 3
  (void)per;
#pragma unroll
  for (int q = 0; q < Sh::kHashMax / (4 * Sh::kThreads); q++) {
    const int j = 4 * (tid + q * Sh::kThreads);
    uint4 k4 = make_uint4(0u, 0u, 0u, 0u), v4 = k4;
    if (j < H) {
      k4 = *reinterpret_cast<const uint4 *>(keys + j);
      v4 = *reinterpret_cast<const uint4 *>(cnts + j);
      *reinterpret_cast<uint4 *>(keys + j) = make_uint4(0u, 0u, 0u, 0u);
      *reinterpret_cast<uint4 *>(cnts + j) = make_uint4(0u, 0u, 0u, 0u);
    }
    const uint32_t kk[4] = {k4.x, k4.y, k4.z, k4.w}, vv[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int i = 4 * q + u;
      ek[i] = ~0u;
      ec[i] = 0u;
      er[i] = 0u;
      if (kk[u] && vv[u]) {
        const uint32_t col = kk[u] - 1u - uint32_t(c0);
        ek[i] = col;
        ec[i] = vv[u];
        rsum += vv[u];
        if (!A.any_order) atomicOr(&L.L1[col >> 10], 1u << ((col >> 5) & 31u));
      }
    }
  }
  __syncthreads();
  STAT_ADD(46, STAT_CLOCK() - c_h0);
  if (A.any_order) {  // COOC_FLAG_ANY_ORDER: the keys in slot order, a thread's after the threads before it
    uint32_t cnt = 0;
#pragma unroll
    for (int i = 0; i < Sh::kHashMax / Sh::kThreads; i++) cnt += ek[i] != ~0u;
    uint32_t ne;
    uint32_t q = block_excl_scan<Sh::kWaves>(cnt, &ne, S_.wtot);
    const unsigned long long c_a1 = STAT_CLOCK();
    STAT_ADD(20, c_a1 - c_h0);
    const int64_t base = sp_reserve<Sh>(A, S_, ne);  // (barrier)
    const unsigned long long c_a2 = STAT_CLOCK();
    STAT_ADD(21, c_a2 - c_a1);
    if (base >= 0 && ne <= uint32_t(Sh::kWStage)) {  // staged in LDS, then 16-B stores (as below)
      uint32_t *sc = keys + Sh::kWStage, *sn = cnts + Sh::kWStage;
#pragma unroll
      for (int i = 0; i < Sh::kHashMax / Sh::kThreads; i++) {
        if (ek[i] == ~0u) continue;
        sc[q] = uint32_t(sp_col(A, uint32_t(c0) + ek[i]));
        sn[q] = ec[i];
        q++;
      }
      __syncthreads();
      const uint32_t head = min(ne, uint32_t((4 - (base & 3)) & 3));
      const uint32_t body = (ne - head) >> 2;
      for (uint32_t j = tid; j < head; j += Sh::kThreads) {
        A.col_out[base + j] = int32_t(sc[j]);
        A.cnt_out[base + j] = sn[j];
      }
      int4 *co4 = reinterpret_cast<int4 *>(A.col_out + base + head);
      uint4 *cn4 = reinterpret_cast<uint4 *>(A.cnt_out + base + head);
      for (uint32_t j = tid; j < body; j += Sh::kThreads) {
        const uint32_t r = head + 4 * j;
        co4[j] = make_int4(int32_t(sc[r]), int32_t(sc[r + 1]), int32_t(sc[r + 2]), int32_t(sc[r + 3]));
        cn4[j] = make_uint4(sn[r], sn[r + 1], sn[r + 2], sn[r + 3]);
      }
      for (uint32_t r = head + 4 * body + tid; r < ne; r += Sh::kThreads) {
        A.col_out[base + r] = int32_t(sc[r]);
        A.cnt_out[base + r] = sn[r];
      }
      __syncthreads();
      for (uint32_t r = tid; r < ne; r += Sh::kThreads) {
        sc[r] = 0u;
        sn[r] = 0u;
      }
    } else if (base >= 0) {
#pragma unroll
      for (int i = 0; i < Sh::kHashMax / Sh::kThreads; i++) {
        if (ek[i] == ~0u) continue;
        if (BCHK(A, base + q < A.cap, 128)) {
          A.col_out[base + q] = sp_col(A, uint32_t(c0) + ek[i]);
          A.cnt_out[base + q] = ec[i];
        }
        q++;
      }
    }
    __syncthreads();
    STAT_ADD(22, STAT_CLOCK() - c_a2);
    STAT_ADD(23, ne);
    return;
  }
  uint32_t nblk;
  {
    static_assert(Sh::kL1Words % Sh::kThreads == 0, "L1 words per thread");
    constexpr int kW = Sh::kL1Words / Sh::kThreads;  // consecutive L1 words per thread
    uint32_t pc[kW], x = 0;
#pragma unroll
    for (int i = 0; i < kW; i++) {
      pc[i] = kW * tid + i < nL1 ? uint32_t(__popc(L.L1[kW * tid + i])) : 0u;
      x += pc[i];
    }
    const uint32_t p = block_excl_scan<Sh::kWaves>(x, &nblk, S_.wtot);
    uint32_t run = p;
#pragma unroll
    for (int i = 0; i < kW; i++) {
      if (kW * tid + i < nL1) L.L1pre[kW * tid + i] = run;
      run += pc[i];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < Sh::kHashMax / Sh::kThreads; i++) {
    if (ek[i] == ~0u) continue;
    const uint32_t col = ek[i], wd = col >> 10, bit = (col >> 5) & 31u;
    const uint32_t r = L.L1pre[wd] + uint32_t(__popc(L.L1[wd] & ((1u << bit) - 1u)));
    er[i] = r;
    atomicOr(&keys[r], 1u << (col & 31u));
  }
  __syncthreads();
  STAT_ADD(47, STAT_CLOCK() - c_h0);
  const uint32_t pb = (nblk + Sh::kThreads - 1) / Sh::kThreads;
  const uint32_t r0 = min(nblk, uint32_t(tid) * pb), r1 = min(nblk, r0 + pb);
  uint32_t local = 0;
  for (uint32_t r = r0; r < r1; r++) local += uint32_t(__popc(keys[r]));
  uint32_t ne;
  uint32_t run = block_excl_scan<Sh::kWaves>(local, &ne, S_.wtot);
  for (uint32_t r = r0; r < r1; r++) {
    cnts[r] = run;
    run += uint32_t(__popc(keys[r]));
  }
  const unsigned long long c_h1 = STAT_CLOCK();
  STAT_ADD(20, c_h1 - c_h0);
  const int64_t base = sp_reserve<Sh>(A, S_, ne);  // (barrier: bases visible)
  const unsigned long long c_h2 = STAT_CLOCK();
  STAT_ADD(21, c_h2 - c_h1);
#ifndef COOC_SP_NO_STAGED_WRITE
  if (base >= 0 && ne <= uint32_t(Sh::kWStage)) {
    // the chunk's entries land in LDS at their sorted positions (the free upper halves of the emptied key
    // and count areas), then leave in order: 16-B stores of whole column / count runs instead of one
    // scattered 4-B store per entry and array
    uint32_t *sc = keys + Sh::kWStage, *sn = cnts + Sh::kWStage;
    // (after a relabel a column maps back by a lookup in tile 0's 64 KB table, a subtraction above)
    const bool hot0 = A.hot_col && c0 < kTW;
    const uint32_t shift = A.hot_col ? uint32_t(kTW) : 0u;
#pragma unroll
    for (int i = 0; i < Sh::kHashMax / Sh::kThreads; i++) {
      if (ek[i] == ~0u) continue;
      const uint32_t col = ek[i], r = er[i];
      const uint32_t q = cnts[r] + uint32_t(__popc(keys[r] & ((1u << (col & 31u)) - 1u)));
      const uint32_t c = uint32_t(c0) + col;
      sc[q] = hot0 && c < uint32_t(kTW) ? uint32_t(A.hot_col[c]) : c - shift;
      sn[q] = ec[i];
    }
    __syncthreads();
    const uint32_t head = min(ne, uint32_t((4 - (base & 3)) & 3));  // entries before the first 16-B boundary
    const uint32_t body = (ne - head) >> 2;
    for (uint32_t j = tid; j < head; j += Sh::kThreads) {
      A.col_out[base + j] = int32_t(sc[j]);
      A.cnt_out[base + j] = sn[j];
    }
    int4 *co4 = reinterpret_cast<int4 *>(A.col_out + base + head);
    uint4 *cn4 = reinterpret_cast<uint4 *>(A.cnt_out + base + head);
    for (uint32_t j = tid; j < body; j += Sh::kThreads) {
      const uint32_t q = head + 4 * j;
      co4[j] = make_int4(int32_t(sc[q]), int32_t(sc[q + 1]), int32_t(sc[q + 2]), int32_t(sc[q + 3]));
      cn4[j] = make_uint4(sn[q], sn[q + 1], sn[q + 2], sn[q + 3]);
    }
    for (uint32_t q = head + 4 * body + tid; q < ne; q += Sh::kThreads) {
      A.col_out[base + q] = int32_t(sc[q]);
      A.cnt_out[base + q] = sn[q];
    }
    __syncthreads();
    for (uint32_t q = tid; q < ne; q += Sh::kThreads) {  // the areas go back to zero for the next chunk
      sc[q] = 0u;
      sn[q] = 0u;
    }
  } else
#endif
  if (base >= 0) {
#pragma unroll
    for (int i = 0; i < Sh::kHashMax / Sh::kThreads; i++) {
      if (ek[i] == ~0u) continue;
      const uint32_t col = ek[i], r = er[i];
      const int64_t pos = base + cnts[r] + uint32_t(__popc(keys[r] & ((1u << (col & 31u)) - 1u)));
      if (BCHK(A, pos >= 0 && pos < A.cap, 128)) {
        A.col_out[pos] = sp_col(A, uint32_t(c0) + col);
        A.cnt_out[pos] = ec[i];
      }
    }
  }
  __syncthreads();
  STAT_ADD(22, STAT_CLOCK() - c_h2);
  STAT_ADD(23, ne);
  for (uint32_t r = tid; r < nblk; r += Sh::kThreads) {
    keys[r] = 0u;
    cnts[r] = 0u;
  }
  for (int32_t i = tid; i < nL1; i += Sh::kThreads) L.L1[i] = 0u;
  __syncthreads();
}

// The workgroup loop.  A work item is a whole row (its chunks in column order, appended to the row's
// contiguous output) or a split row's (tile, contribution share), added into the staging row.  One
// code path for every chunk kind, so that the walk and the two compactions exist once.
// The shape (SpBig: 512 threads, two workgroups per CU; SpMid: 256 threads, four per CU) fixes the LDS layout;
// both keep 4 waves per SIMD (<= 128 VGPRs).  A launch takes the queue range [A.q_begin, A.q_end).
template <class Sh>
__global__ __launch_bounds__(Sh::kThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_sp_main(SpArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ SpStatic S_;
  SpShared L;
  L.R = lds;
  L.L1 = L.R + Sh::kRWords;
  L.L1pre = L.L1 + Sh::kL1Words;
  L.gb = reinterpret_cast<int32_t *>(L.L1pre + Sh::kL1Words);
  L.info = reinterpret_cast<uint32_t *>(L.gb + Sh::kDb);
  L.vst = L.info + Sh::kDb;
  L.qstart = reinterpret_cast<int32_t *>(L.vst + Sh::kDb + 4);
  const int tid = threadIdx.x;
  for (int32_t i = tid; i < Sh::kRWords + Sh::kL1Words; i += Sh::kThreads) L.R[i] = 0u;
  if (tid == 0) {
    S_.slab_cur = S_.slab_end = 0;
    S_.flag = 0u;
  }
  // (the queue's tail: the mid rows (the mid shape's launch), the small rows (k_sp_small), the tiny ones (k_sp_tiny))
  const int64_t n_work = A.q_end - A.q_begin;
#ifdef COOC_SP_STATS
  if (threadIdx.x < 64) S_.st[threadIdx.x] = 0ull;
  const unsigned long long t_start = STAT_CLOCK();
#endif
  if (tid == 0) S_.work = atomicAdd(A.qctr, 1);
  __syncthreads();
  uint64_t rsum = 0;  // this thread's share of the current whole row's count sum
  for (;;) {
    const int32_t w = uni(S_.work);
    if (w >= n_work) break;
    // the next item is dequeued now and read at the end of this one (its latency hides behind the work)
    uint32_t next = 0;
    if (tid == 0) next = atomicAdd(A.qctr, 1);
    const SpWork it = A.queue[A.q_begin + w];
    const int32_t a = it.row;
    const int32_t ra = sp_rank(A, a);  // the row's own column (the self term), in column-rank space
    const bool split = it.kind == -2;  // a share of a split row's contributions, every tile, into staging
    const int64_t k0 = it.k0, k1 = it.k1;
    int t = 0;
    const int t_end = A.T;
    const uint64_t st = it.st, dn = it.dn, hz0 = it.hz[0], hz1 = it.hz[1];
    // gather mode (rows with many chunks, split shares): the lists are walked once; tile 0 is counted
    // on the way and every other tile's groups go to a bucket that its chunk then reads contiguously
    // (instead of one walk of every contribution per chunk).  Off when the tails exceed the scratch.
    bool gather = A.scr_cap > 0 && it.gslot >= 0;
    if (!split && tid == 0) {
      // a row expected to fill much of a slab gets a region of its own (est + 1/8), so it neither
      // moves nor strands the workgroup's slab; the slab is resumed after it
      const int64_t e = it.est;
      S_.own = 0u;
      if (e > A.slab / 4 && e + e / 8 > S_.slab_end - S_.slab_cur) {
        const int64_t take = e + e / 8 + 1024;
        const int64_t b = int64_t(atomicAdd(A.bump, (unsigned long long)take));
        if (b + take <= A.cap) {
          S_.saved_cur = S_.slab_cur;
          S_.saved_end = S_.slab_end;
          S_.own = 1u;
          S_.slab_cur = b;
          S_.slab_end = b + take;
        }
      }
      S_.row_begin = S_.slab_cur;
      S_.row_n = 0;
      S_.rsum = 0ull;
    }
    // the closed-form row sum this row's counts must add up to (read now, compared at the end)
    const int64_t rs_expect = (!split && tid == 0) ? A.rowsum[a] : 0;
    bool rs_expect_ok = false;
    if (gather && tid < 64) {
      // bucket capacity of tile t >= 1 (in ids): the item's expected ids in tile t, Wi g_t, + 10% + 64.
      // A bucket that still overflows only sends its tile's chunk back to walking the lists.
      const float Wi = float(A.epre[k1] - A.epre[k0]);
      uint32_t cap = 0;
      if (tid >= 1 && tid < A.T) cap = (uint32_t(1.1f * Wi * A.gmass[tid]) + 64u + 3u) & ~3u;  // ids, 16-B aligned
      const uint32_t inc = wave_incl_scan(cap);
      if (tid < A.T) {
        S_.bstart[tid] = inc - cap;
        S_.bcur[tid] = 0u;
      }
      if (tid == A.T - 1) S_.bstart[A.T] = inc;
    }
    __syncthreads();
    gather = gather && uni(S_.bstart[A.T]) <= uint32_t(A.scr_cap) * 4u;
    const int dense_until = split ? t_end : -1;  // tiles below it go dense (split items)
    int32_t H = 0;                               // 0: table size from the estimate
    // a whole row whose hash table overflows (more distinct keys than the planner expected) is handed to
    // the sort + segmented-reduce path (k_sr_*, after this kernel) whole: its entries so far are dropped
    bool deferred = !split && A.sort_all;
    if (deferred) t = t_end;
    while (t < t_end) {
      // ---- this chunk: tiles [t, t1), dense or hash
      const bool dense = t < dense_until || ((dn >> t) & 1ull);
      int t1 = t + 1;
      if (!dense) {
        const uint64_t rest = t + 1 < 64 ? st >> (t + 1) : 0ull;
        t1 = rest ? min(t_end, t + __ffsll((long long)rest)) : t_end;
        if (H == 0) H = min(Sh::kHashMax, kHashMin << (((t < 32 ? hz0 : hz1) >> (2 * (t & 31))) & 3u));  // the planner's size
      }
      const int32_t c0 = t * kTW, c1 = min(A.M, t1 * kTW);
      WalkOp op;
      op.mode = dense ? 0 : 1;
      op.c0 = uint32_t(c0);
      const uint32_t lg = dense ? 0u : 31u - uint32_t(__clz(uint32_t(H)));
      op.hshift = 32u - lg;
      op.hmask = uint32_t(H) - 1u;
      if (tid == 0) {
        S_.flag = 0u;
      }
      __syncthreads();
      const unsigned long long c_walk = STAT_CLOCK();
      op.sbase = int64_t(blockIdx.x) * A.scr_cap;
      uint64_t walked;
      if (gather && t == 0) {  // tile 0 (a dense chunk) counted, the other tiles' groups to their buckets
        op.mode = 2;
        walked = sp_walk<Sh>(A, L, S_, k0, k1, 0, A.T, true, op);
        if (tid < 64) {
          const bool o = tid >= 1 && tid < A.T && S_.bcur[tid] > S_.bstart[tid + 1] - S_.bstart[tid];
          const uint64_t m = __ballot(o);
          if (tid == 0) S_.ovf = m;
        }
        sp_global_sync();  // the buckets are read back by other waves (and this item's lines are new)
      } else if (gather && !(uint64_t(uni(int64_t(S_.ovf))) & (((t1 < 64 ? (1ull << t1) : 0ull) - 1ull) & ~((1ull << t) - 1ull)))) {
        // a gathered tile range: the filled parts of its tiles' buckets, walked as one batch
        const int nb = t1 - t;
        const uint32_t bs = tid < nb ? S_.bstart[t + tid] : 0u;
        const uint32_t be = tid < nb ? bs + S_.bcur[t + tid] : 0u;
        walked = sp_walk_batch<Sh, 4>(A, L, S_, A.scratch + op.sbase, A.scr_cap, nb, bs, be, op);
      } else {  // (also a gathered chunk whose bucket overflowed)
        walked = sp_walk<Sh>(A, L, S_, k0, k1, t, t1, !split && t == 0 && t1 == A.T, op);
      }
      const unsigned long long c_walked = STAT_CLOCK();
      STAT_ADD(split ? 4 : dense ? 0 : 1, c_walked - c_walk);
#ifdef COOC_SP_STATS
      // hash chunk classes: 0 = a light row (one hash chunk over every tile), 1 = a gathered tile range
      // (buckets), 2 = any other (walks the lists over its tile range)
      const int hcls = (!split && t == 0 && t1 == t_end) ? 0 : (gather && t > 0) ? 1 : 2;
      if (!dense && !split) {
        STAT_ADD(28 + 6 * hcls, 1);
        STAT_ADD(29 + 6 * hcls, c_walked - c_walk);
        STAT_ADD(31 + 6 * hcls, walked);
        STAT_ADD(33 + 6 * hcls, k1 - k0);
      }
#endif
      STAT_ADD(dense ? 9 : 10, walked);
      STAT_ADD(dense ? 5 : 6, 1);
      if (!dense && uni(S_.flag)) {
        STAT_ADD(7, 1);
        // overflow: clear the table (and the gather walk's state is this item's only); the row is deferred
        for (int32_t j = tid; j < H; j += Sh::kThreads) {
          L.R[j] = 0u;
          L.R[Sh::kHashMax + j] = 0u;
        }
        deferred = true;
        __syncthreads();  // every wave has read the flag and cleared its slots
        break;
      }
      // the -1 at column a per contribution whose walk includes its own position (whole rows)
      const uint32_t self = uint32_t(A.spre ? A.spre[k1] - A.spre[k0] : k1 - k0);
      if (split) {
        uint32_t *dst = A.staging + int64_t(A.split_slot[a]) * A.sstride + c0;
        if (!Sh::kU16) {  // (split rows are never mid rows)
          for (int32_t i = tid; i < c1 - c0; i += Sh::kThreads) {
            const uint32_t v = L.R[i];
            if (v) {
              atomicAdd(dst + i, v);
              L.R[i] = 0u;
            }
          }
        }
        __syncthreads();
        STAT_ADD(26, STAT_CLOCK() - c_walked);  // the share's flush of this tile into the staging row
      } else if (dense) {
        if (tid == 0 && ra >= c0 && ra < c1) {
          const uint32_t o = uint32_t(ra - c0);  // (the counter holds >= self: no borrow into the other u16)
          if (Sh::kU16)
            L.R[o >> 1] -= self << ((o & 1u) << 4);
          else
            L.R[o] -= self;
        }
        __syncthreads();
        sp_dense_compact<Sh>(A, L, S_, c1 - c0, c0, rsum);
        STAT_ADD(2, STAT_CLOCK() - c_walked);
      } else {
        if (tid == 0 && ra >= c0 && ra < c1) {
          uint32_t h = (uint32_t(ra) * 0x9E3779B1u) >> op.hshift;
          for (int p = 0; p < H; p++) {
            if (L.R[h] == uint32_t(ra) + 1u) {
              L.R[Sh::kHashMax + h] -= self;
              break;
            }
            h = (h + 1u) & op.hmask;
          }
        }
        __syncthreads();
        sp_hash_compact<Sh>(A, L, S_, H, c0, c1, rsum);
        STAT_ADD(3, STAT_CLOCK() - c_walked);
#ifdef COOC_SP_STATS
        STAT_ADD(30 + 6 * hcls, STAT_CLOCK() - c_walked);
        STAT_ADD(32 + 6 * hcls, uni(S_.row_n));
#endif
        STAT_ADD(14, H);
      }
      t = t1;
      H = 0;
    }
    STAT_ADD(split ? 12 : 11, 1);
    if (deferred) {
      STAT_ADD(8, 1);
      rsum = 0;
      if (tid == 0) {
        A.deferred[atomicAdd(reinterpret_cast<unsigned long long *>(&A.tot->n_deferred), 1ull)] = a;
        // the row's entries so far are abandoned: at the tail of the workgroup's slab they are handed back
        // (a row region of its own is restored below and its space stays unused)
        if (!S_.own) S_.slab_cur = S_.row_begin;
        S_.row_n = 0;
      }
    }
    if (!split) {  // the row-sum check: every count of the row, summed exactly (u64), == W_a - c_a
      for (int o = 32; o > 0; o >>= 1) rsum += __shfl_xor(rsum, o, 64);
      if ((tid & 63) == 0 && rsum) atomicAdd(&S_.rsum, (unsigned long long)rsum);
    }
    rsum = 0;
    if (!split && tid == 0) {
      A.row_base[a] = S_.row_n ? S_.row_begin : 0;
      A.row_nnz[a] = int32_t(S_.row_n);
      if (S_.own) {
        S_.slab_cur = S_.saved_cur;
        S_.slab_end = S_.saved_end;
      }
    }
    if (tid == 0) S_.work = next;
    __syncthreads();
    // a uint32 counter that wrapped, or any id lost or counted twice, breaks the sum
#ifdef COOC_SP_STATS
    if (A.exp) rs_expect_ok = true;  // (experiments drop ids on purpose)
#endif
    if (!split && !deferred && !rs_expect_ok && tid == 0 && S_.rsum != (unsigned long long)rs_expect) {
      atomicOr(reinterpret_cast<unsigned long long *>(&A.tot->err), 2ull);
      A.tot->bad_row = a;
    }
  }
#ifdef COOC_SP_STATS
  if (tid == 0) {
    S_.st[13] = STAT_CLOCK() - t_start;
    for (int k = 0; k < 64; k++) atomicAdd(A.stats + k, S_.st[k]);
  }
#endif
}

// Split rows: the staging row (self term applied on the fly) compacted in column order into an
// exact-size region; the uint32 overflow check compares the count sum with the closed-form row sum.
// One 1,024-thread block per row; staging rows have a 16-B aligned stride, so every lane reads
// kFinU x 4 counters (16-B loads) per step and the waves own 4,096-column-aligned ranges.
constexpr int kFinThreads = 1024, kFinWaves = kFinThreads / 64, kFinU = 4;
__global__ __launch_bounds__(kFinThreads) void k_sp_split_finalize(const int32_t *__restrict__ split_row,
                                                                    const uint32_t *__restrict__ staging, int64_t stride,
                                                                    int32_t M, const int64_t *__restrict__ row_ptr,
                                                                    const int64_t *__restrict__ rowsum,
                                                                    int32_t *__restrict__ col_out,
                                                                    uint32_t *__restrict__ cnt_out,
                                                                    unsigned long long *__restrict__ bump, int64_t cap,
                                                                    int64_t *__restrict__ row_base,
                                                                    int32_t *__restrict__ row_nnz,
                                                                    PlanTotals *__restrict__ tot,
                                                                    const int64_t *__restrict__ spre,
                                                                    const int32_t *__restrict__ hot_col,
                                                                    const int32_t *__restrict__ pos_of) {
  __shared__ uint32_t s_w[kFinWaves];
  __shared__ uint64_t s_red[kFinWaves];
  __shared__ int64_t s_base;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int32_t s = blockIdx.x;
  const int32_t a = split_row[s];
  const int32_t ra = relabel_pos(pos_of, uint32_t(a));  // staging rows are in relabelled column space
  const uint32_t self = uint32_t(spre ? spre[row_ptr[a + 1]] - spre[row_ptr[a]] : row_ptr[a + 1] - row_ptr[a]);
  const uint32_t *row = staging + int64_t(s) * stride;
  constexpr int32_t kStep = 64 * 4 * kFinU;  // columns per wave step
  const int32_t per = ((M + kFinWaves - 1) / kFinWaves + kStep - 1) / kStep * kStep;
  const int32_t lo = min(M, wave * per), hi = min(M, lo + per);
  auto load = [&](int32_t b, uint32_t v[4]) {
    if (b + 3 < hi) {
      const uint4 q = *reinterpret_cast<const uint4 *>(row + b);
      v[0] = q.x;
      v[1] = q.y;
      v[2] = q.z;
      v[3] = q.w;
    } else {
      for (int k = 0; k < 4; k++) v[k] = b + k < hi ? row[b + k] : 0u;
    }
    for (int k = 0; k < 4; k++)
      if (b + k == ra) v[k] -= self;
  };
  uint32_t cnt = 0;
  uint64_t sum = 0;
  for (int32_t b0 = lo; b0 < hi; b0 += kStep) {
    uint32_t v[kFinU][4];
#pragma unroll
    for (int u = 0; u < kFinU; u++) load(b0 + (u * 64 + lane) * 4, v[u]);
#pragma unroll
    for (int u = 0; u < kFinU; u++)
#pragma unroll
      for (int k = 0; k < 4; k++) {
        cnt += v[u][k] != 0u;
        sum += v[u][k];
      }
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if (lane == 0) s_w[wave] = cnt;
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  if (lane == 0) s_red[wave] = sum;
  __syncthreads();
  uint32_t off = 0, tot_n = 0;
  uint64_t total_sum = 0;
  for (int w = 0; w < kFinWaves; w++) {
    off += w < wave ? s_w[w] : 0u;
    tot_n += s_w[w];
    total_sum += s_red[w];
  }
  if (tid == 0) {
    int64_t b = int64_t(atomicAdd(bump, (unsigned long long)tot_n));
    if (b + int64_t(tot_n) > cap) {
      atomicOr(reinterpret_cast<unsigned long long *>(&tot->err), 4ull);
      b = -1;
    }
    s_base = b;
    row_base[a] = b < 0 ? 0 : b;
    row_nnz[a] = int32_t(tot_n);
    if (total_sum != uint64_t(rowsum[a])) atomicOr(reinterpret_cast<unsigned long long *>(&tot->err), 2ull);
  }
  __syncthreads();
  const int64_t base = s_base;
  if (base < 0) return;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int32_t b0 = lo; b0 < hi; b0 += kStep) {
    uint32_t v[kFinU][4];
#pragma unroll
    for (int u = 0; u < kFinU; u++) load(b0 + (u * 64 + lane) * 4, v[u]);
#pragma unroll
    for (int u = 0; u < kFinU; u++) {
      const int32_t b = b0 + (u * 64 + lane) * 4;
      const uint32_t c = (v[u][0] != 0u) + (v[u][1] != 0u) + (v[u][2] != 0u) + (v[u][3] != 0u);
      const uint64_t m0 = __ballot(c & 1u), m1 = __ballot(c & 2u), m2 = __ballot(c & 4u);
      int64_t pos = base + off + uint32_t(__popcll(m0 & lt_mask)) + 2u * uint32_t(__popcll(m1 & lt_mask)) +
                    4u * uint32_t(__popcll(m2 & lt_mask));
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (v[u][k]) {
          col_out[pos] = relabel_col(hot_col, uint32_t(b + k));
          cnt_out[pos] = v[u][k];
          pos++;
        }
      off += uint32_t(__popcll(m0)) + 2u * uint32_t(__popcll(m1)) + 4u * uint32_t(__popcll(m2));
    }
  }
}

__global__ void k_sp_nnz_total(const int32_t *__restrict__ row_nnz, int32_t M, PlanTotals *__restrict__ tot) {
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

__global__ void k_sp_reset_run(PlanTotals *__restrict__ tot, int32_t *__restrict__ qctr,
                               unsigned long long *__restrict__ bump) {
  tot->err &= ~int64_t(6);  // the region (4) and row-sum (2) checks of the previous attempt
  tot->nnz_total = 0;
  tot->n_deferred = 0;
  tot->tiny_ctr = 0;
  tot->small_ctr = 0;
  qctr[0] = qctr[1] = 0;
  bump[0] = 0;
}

// ---- the sort + segmented-reduce path (rows whose LDS hash table overflowed; COOC_FLAG_SORT_ROWS: all) ----
// The north star's overflow fallback for the per-row Int2ShortOpenHashMap (ItemRowAggregator.java:21-31):
// every pair of the deferred rows becomes one packed 64-bit key (row slot << 32 | partner id), the keys
// are radix-sorted (hipCUB onesweep: wave-level digit ranking in LDS), runs of equal keys are counted
// (DeviceRunLengthEncode: the segmented reduce of the +1 increments) and each row's runs are written as
// its padded-CSR slice, in column order, with the same row-sum check as k_sp_main.  Deferred rows are
// processed in batches of at most kSrBatchPairs pairs.
constexpr int kSrThreads = 256;

// One workgroup per deferred row of the batch: every contribution's list (its tile-0 ids from arena0,
// the rest from arena1) appended to the row's key range at kbase[j] + (epre[k] - epre[k0]).
__global__ __launch_bounds__(kSrThreads) void k_sr_expand(const int32_t *__restrict__ rows, const int64_t *__restrict__ kbase,
                                                          const int64_t *__restrict__ row_ptr,
                                                          const int64_t *__restrict__ epre,
                                                          const uint32_t *__restrict__ vals, const int32_t *__restrict__ tb,
                                                          const uint16_t *__restrict__ arena0,
                                                          const uint32_t *__restrict__ arena1, int32_t T,
                                                          uint64_t *__restrict__ keys) {
  const int j = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int32_t a = rows[j];
  const int64_t k0 = row_ptr[a], k1 = row_ptr[a + 1], e0 = epre[k0];
  const uint64_t tag = uint64_t(j) << 32;
  for (int64_t k = k0 + wave; k < k1; k += kSrThreads / 64) {
    const uint32_t u = vals[k] & kListMask;
    const int32_t *tbu = tb + int64_t(u) * (T + 2);
    const int32_t s0 = tbu[0], n0 = tbu[T + 1] - s0, s1 = tbu[1], n1 = tbu[T] - s1;
    uint64_t *o = keys + kbase[j] + (epre[k] - e0);
    for (int32_t q = lane; q < n0; q += 64) o[q] = tag | uint32_t(arena0[s0 + q]);
    for (int32_t q = lane; q < n1; q += 64) o[n0 + q] = tag | arena1[s1 + q];
  }
}

// First run of every row slot j of the batch (runs are sorted by (slot, column)): rstart[j] = lower bound
// of j << 32 in the run keys; rstart[nb] = the run count.
__global__ void k_sr_bounds(const uint64_t *__restrict__ ukeys, const int64_t *__restrict__ n_runs_p, int32_t nb,
                            int64_t *__restrict__ rstart) {
  const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j > nb) return;
  const int64_t n = *n_runs_p;
  int64_t lo = 0, hi = n;
  const uint64_t key = uint64_t(j) << 32;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (ukeys[mid] < key) lo = mid + 1; else hi = mid;
  }
  rstart[j] = lo;
}

// One workgroup per row slot: the row's runs -> (column, count) entries in column order at an exactly
// sized bump reservation; the diagonal run loses the row's self term (and is dropped at zero); the counts
// must add up to the closed-form row sum (err bit 1 with bad_row otherwise, as in k_sp_main).
__global__ __launch_bounds__(kSrThreads) void k_sr_emit(const int32_t *__restrict__ rows, const int64_t *__restrict__ rstart,
                                                        const uint64_t *__restrict__ ukeys,
                                                        const uint32_t *__restrict__ ucnt,
                                                        const int64_t *__restrict__ row_ptr,
                                                        const int64_t *__restrict__ spre,
                                                        const int64_t *__restrict__ rowsum,
                                                        int32_t *__restrict__ col_out, uint32_t *__restrict__ cnt_out,
                                                        unsigned long long *__restrict__ bump, int64_t cap,
                                                        int64_t *__restrict__ row_base, int32_t *__restrict__ row_nnz,
                                                        PlanTotals *__restrict__ tot, const int32_t *__restrict__ hot_col,
                                                        const int32_t *__restrict__ pos_of) {
  __shared__ int64_t s_diag, s_base;
  __shared__ unsigned long long s_sum;
  const int j = blockIdx.x, tid = threadIdx.x;
  const int32_t a = rows[j];
  const uint32_t ra = uint32_t(relabel_pos(pos_of, uint32_t(a)));  // the keys' columns are relabelled
  const int64_t r0 = rstart[j], r1 = rstart[j + 1];
  const int64_t k0 = row_ptr[a], k1 = row_ptr[a + 1];
  const uint32_t self = uint32_t(spre ? spre[k1] - spre[k0] : k1 - k0);
  if (tid == 0) {
    s_diag = -1;
    s_sum = 0ull;
  }
  __syncthreads();
  uint64_t sum = 0;
  for (int64_t r = r0 + tid; r < r1; r += kSrThreads) {
    sum += ucnt[r];
    if (uint32_t(ukeys[r]) == ra) s_diag = r;
  }
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  if ((tid & 63) == 0) atomicAdd(&s_sum, (unsigned long long)sum);
  __syncthreads();
  const int64_t diag = s_diag;
  const bool drop = diag >= 0 && ucnt[diag] == self;
  const int64_t n = (r1 - r0) - (drop ? 1 : 0);
  if (tid == 0) {
    int64_t b = n > 0 ? int64_t(atomicAdd(bump, (unsigned long long)n)) : 0;
    if (b + n > cap) {
      atomicOr(reinterpret_cast<unsigned long long *>(&tot->err), 4ull);
      b = -1;
    }
    s_base = b;
    row_base[a] = b < 0 ? 0 : b;
    row_nnz[a] = b < 0 ? 0 : int32_t(n);
    // self pairs are part of the sums of the runs; a diagonal run below the self term is an error too
    if (s_sum != (unsigned long long)(rowsum[a] + self) || (self && (diag < 0 || ucnt[diag] < self))) {
      atomicOr(reinterpret_cast<unsigned long long *>(&tot->err), 2ull);
      tot->bad_row = a;
    }
  }
  __syncthreads();
  const int64_t base = s_base;
  if (base < 0) return;
  for (int64_t r = r0 + tid; r < r1; r += kSrThreads) {
    if (drop && r == diag) continue;
    const int64_t q = base + (r - r0) - (drop && r > diag ? 1 : 0);
    col_out[q] = relabel_col(hot_col, uint32_t(ukeys[r]));
    cnt_out[q] = ucnt[r] - (r == diag ? self : 0u);
  }
}

// One contribution's list -- n0 tile-0 ids of arena0 at s0 (a multiple of 8), then n1 other ids of arena1
// at s1 (a multiple of 4): the user's parts are 16-B aligned -- copied by one wave to d[0, n0 + n1): 16-B
// loads (8 or 4 ids), both parts' loads of a step issued before their stores.
__device__ inline void wave_copy_list(const uint16_t *__restrict__ a0, const uint32_t *__restrict__ a1, uint32_t s0,
                                      uint32_t n0, uint32_t s1, uint32_t n1, uint32_t *d, int lane) {
  const uint4 *p0 = reinterpret_cast<const uint4 *>(a0 + s0);
  const uint4 *p1 = reinterpret_cast<const uint4 *>(a1 + s1);
  const uint32_t g0 = (n0 + 7u) >> 3, g1 = (n1 + 3u) >> 2, g = max(g0, g1);
  for (uint32_t q = uint32_t(lane); q < g; q += 64u) {
    uint4 v0 = make_uint4(0u, 0u, 0u, 0u), v1 = v0;
    if (q < g0) v0 = p0[q];
    if (q < g1) v1 = p1[q];
    if (q < g0) {
      const uint32_t w[4] = {v0.x, v0.y, v0.z, v0.w};
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const uint32_t pos = 8u * q + uint32_t(i);
        if (pos < n0) d[pos] = (w[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
      }
    }
    if (q < g1) {
      const uint32_t w[4] = {v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t pos = 4u * q + uint32_t(i);
        if (pos < n1) d[n0 + pos] = w[i];
      }
    }
  }
}

// ---- small rows: one 512-thread workgroup per row -----------------------------------------------------
// A whole row of kTinyW < W <= kSmallW pairs -- at C3 the half million rows of the Zipf tail, each one LDS
// hash chunk over every tile in k_sp_main (~20 us per chunk there, two chunks per CU) -- sorted instead: its
// lists gathered into 16 KB of LDS (a wave per contribution, coalesced), LSD-radix-sorted by the workgroup
// (7-bit digits, wave ballots rank equal digits), equal columns counted (the segmented reduce of the +1
// increments), the diagonal's self term removed, the entries written in column order from a
// per-workgroup output slab.  At 33 KB per workgroup a CU holds four rows in flight.
constexpr int kSmallThreads = 512, kSmallWaves = kSmallThreads / 64;
constexpr int64_t kSmallSlab = 16384;  // output entries reserved per workgroup at a time
constexpr int kRadixBits = 7;

// Stable LSD radix sort of k[0, n), n <= kSmallW, keys < 2^bits, kRadixBits per pass, ping-ponging between
// k and t; returns the buffer that holds the sorted keys.  Wave w owns positions [w P, (w + 1) P),
// P = 64 ceil(n / (64 kWaves)) <= kSmallW / kWaves, 64 at a time: a lane's rank among equal digits is the popcount of the ballot
// match below it plus the wave's running count h[digit][w]; one exclusive scan over (digit, wave) turns
// the counts into the scatter bases.  Four LDS accesses per key per pass.
template <int kThreads>
__device__ uint32_t *block_radix_sort(uint32_t *k, uint32_t *t, uint16_t *h, uint32_t *s_wt, uint32_t n, int bits) {
  constexpr int kWaves = kThreads / 64, kE = kSmallW / kThreads, kD = 1 << kRadixBits;
  static_assert(kD * kWaves == 2 * kThreads, "two scan entries per thread");
  // a wave ranks kE * 64 positions: the rank (< kE * 64 <= 512, 9 bits) and the digit (7 bits) fill all 16 bits,
  // so no 16-bit value is free to mark "no key" -- a position holds a key iff it is below n (checked by position
  // in the scatter; the former 0xffff marker was also digit 127 at rank 511, and that key was never scattered)
  static_assert(kE * 64 <= 512 && kRadixBits <= 7, "rank and digit pack into 16 bits");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t below_mask = (1ull << lane) - 1ull;
  // wave w ranks the span [w P, (w + 1) P) ∩ [0, n): P the smallest multiple of 64 that covers n with every
  // wave (a row of 1,500 keys: 192 positions per wave, not 512 for the first three waves and none for the rest)
  const uint32_t P = ((n + uint32_t(kWaves * 64) - 1u) / uint32_t(kWaves * 64)) * 64u;
  const uint32_t base = uint32_t(wave) * P, lim = min(n, base + P);
  for (int sh = 0; sh < bits; sh += kRadixBits) {
    reinterpret_cast<uint32_t *>(h)[tid] = 0u;
    __syncthreads();
    uint32_t pk[kE / 2];  // (digit << 9 | rank), two per register; meaningful only at positions below n
#pragma unroll
    for (int e = 0; e < kE / 2; e++) pk[e] = 0u;
#pragma unroll
    for (int e = 0; e < kE; e++) {
      const uint32_t p0 = base + uint32_t(e) * 64u;
      if (p0 >= lim) continue;  // (wave-uniform)
      const uint32_t p = p0 + uint32_t(lane);
      const bool v = p < lim;
      const uint32_t d = v ? (k[p] >> sh) & uint32_t(kD - 1) : 0u;
      uint64_t m = __ballot(v);
#pragma unroll
      for (int b = 0; b < kRadixBits; b++) {
        const uint64_t bb = __ballot(v && ((d >> b) & 1u));
        m &= ((d >> b) & 1u) ? bb : ~bb;
      }
      if (v) {
        uint16_t *hd = h + d * kWaves + uint32_t(wave);
        const uint32_t old = *hd, below = uint32_t(__popcll(m & below_mask));
        const uint32_t sh16 = (e & 1) * 16;
        pk[e / 2] = (pk[e / 2] & ~(0xffffu << sh16)) | (((old + below) | (d << 9)) << sh16);
        if (below == 0u) *hd = uint16_t(old + uint32_t(__popcll(m)));  // the group's first lane
      }
    }
    __syncthreads();
    const uint32_t h0 = h[2 * tid], h1 = h[2 * tid + 1];
    const uint32_t inc = wave_incl_scan(h0 + h1);
    if (lane == 63) s_wt[wave] = inc;
    __syncthreads();
    uint32_t ex = inc - h0 - h1;
#pragma unroll
    for (int w = 0; w < kWaves; w++) ex += w < wave ? s_wt[w] : 0u;
    h[2 * tid] = uint16_t(ex);
    h[2 * tid + 1] = uint16_t(ex + h0);
    __syncthreads();
#pragma unroll
    for (int e = 0; e < kE; e++) {
      const uint32_t p = base + uint32_t(e) * 64u + uint32_t(lane);
      if (p >= lim) continue;
      const uint32_t x = (pk[e / 2] >> ((e & 1) * 16)) & 0xffffu, d = x >> 9;
      t[uint32_t(h[d * kWaves + uint32_t(wave)]) + (x & 511u)] = k[p];
    }
    __syncthreads();
    uint32_t *x = k;
    k = t;
    t = x;
  }
  return k;
}

__global__ __launch_bounds__(kSmallThreads) __attribute__((amdgpu_waves_per_eu(8))) void k_sp_small(SpArgs A) {
  __shared__ uint32_t b0[kSmallW + 1], b1[kSmallW + 1];  // (+1: the run starts' end marker)
  __shared__ uint16_t s_h[(1 << kRadixBits) * kSmallWaves];
  __shared__ uint32_t s_wt[kSmallWaves];
  __shared__ int64_t s_i, s_pos, s_cur, s_end;
  __shared__ unsigned long long s_sum;
  __shared__ int32_t s_drop;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t first = A.tot->n_chunks - A.tot->n_tiny - A.tot->n_small, n_small = A.tot->n_small;
  const uint16_t *a0 = reinterpret_cast<const uint16_t *>(A.tarena0);
  const uint32_t *a1 = reinterpret_cast<const uint32_t *>(A.tarena);
  int bits = 1;
  while (bits < 32 && (uint32_t(A.M) - 1u) >> bits) bits++;
  if (tid == 0) s_cur = s_end = 0;
  for (;;) {
    if (tid == 0) {
      s_i = int64_t(atomicAdd(reinterpret_cast<unsigned long long *>(&A.tot->small_ctr), 1ull));
      s_sum = 0ull;
      s_drop = -1;
    }
    __syncthreads();
    const int64_t i = uni(s_i);
    if (i >= n_small) break;
    if (!SP_CHECK(A, first + i >= 0 && first + i < A.tot->n_chunks)) break;
    const SpWork it = A.queue[first + i];
    const int32_t a = it.row;
    if (!SP_CHECK(A, a >= 0 && a < A.M && it.k0 >= 0 && it.k0 < it.k1 && it.k1 <= A.n_contrib)) continue;
    const uint32_t ra = uint32_t(sp_rank(A, a));
    const int64_t k0 = it.k0, k1 = it.k1, e0 = A.epre[k0];
    const int64_t W64 = uni(int64_t(A.epre[k1] - e0));
    // the planner sends rows of kTinyW < W <= kSmallW pairs here; a larger W would overrun the LDS buffers
    // (as k_sp_tiny, the row is refused and the run fails its row-sum check instead)
    if (W64 > int64_t(kSmallW) || W64 <= 0) {
      if (tid == 0) {
        atomicOr(reinterpret_cast<unsigned long long *>(&A.tot->err), 2ull | 8ull);
        A.tot->bad_row = a;
        A.row_nnz[a] = 0;
      }
      __syncthreads();
      continue;
    }
    const uint32_t W = uint32_t(W64);
    const uint32_t self = uint32_t(A.spre ? A.spre[k1] - A.spre[k0] : k1 - k0);
    // 1. the lists at their prefix positions (epre), a wave per contribution: wave w's contributions are
    //    k0 + w + 8 j; lane j reads the j-th one's list bounds (all in one round of loads), then the wave
    //    copies the lists one after another (wave_copy_list)
    for (int64_t kb = k0 + wave; kb < k1; kb += int64_t(kSmallWaves) * 64) {
      const int64_t km = kb + int64_t(kSmallWaves) * lane;
      uint32_t m_s0 = 0, m_n0 = 0, m_s1 = 0, m_n1 = 0, m_d = 0;
      if (km < k1) {
        const uint32_t u = A.vals[km] & kListMask;
        const int32_t *tbu = A.tb + int64_t(SP_CHECK(A, u < A.n_users) ? u : 0u) * (A.T + 2);
        m_s0 = uint32_t(tbu[0]);
        m_n0 = uint32_t(tbu[A.T + 1]) - m_s0;
        m_s1 = uint32_t(tbu[1]);
        m_n1 = uint32_t(tbu[A.T]) - m_s1;
        m_d = uint32_t(A.epre[km] - e0);
        // the list lands inside the row's W ids; its 16-B groups inside the arenas
        if (!SP_CHECK(A, m_d + m_n0 + m_n1 <= W && (int64_t(m_s0) + m_n0 + 7) / 8 <= A.n_groups0 &&
                             (int64_t(m_s1) + m_n1 + 3) / 4 <= A.n_groups))
          m_n0 = m_n1 = 0;
      }
      const int cnt = int(min<int64_t>(64, (k1 - kb + kSmallWaves - 1) / kSmallWaves));
      for (int j = 0; j < cnt; j++)
        wave_copy_list(a0, a1, uint32_t(__shfl(int(m_s0), j, 64)), uint32_t(__shfl(int(m_n0), j, 64)),
                       uint32_t(__shfl(int(m_s1), j, 64)), uint32_t(__shfl(int(m_n1), j, 64)),
                       b0 + uint32_t(__shfl(int(m_d), j, 64)), lane);
    }
    __syncthreads();
    // 2. radix sort
    const uint32_t *b = block_radix_sort<kSmallThreads>(b0, b1, s_h, s_wt, W, bits);
    // 3. runs: the heads (a column's first position) among thread tid's kPer positions, ranked by a block
    //    scan; their positions go to the free buffer (st), then a thread per run
    uint32_t *st = (b == b0) ? b1 : b0;
    constexpr int kPer = kSmallW / kSmallThreads;
    uint32_t hm = 0;
#pragma unroll
    for (int e = 0; e < kPer; e++) {
      const uint32_t p = uint32_t(tid) * kPer + uint32_t(e);
      if (p < W && (p == 0 || b[p] != b[p - 1])) hm |= 1u << e;
    }
    const uint32_t inc = wave_incl_scan(uint32_t(__popc(hm)));
    if (lane == 63) s_wt[wave] = inc;
    __syncthreads();
    uint32_t r = inc - uint32_t(__popc(hm)), n_runs = 0;
#pragma unroll
    for (int w = 0; w < kSmallWaves; w++) {
      r += w < wave ? s_wt[w] : 0u;
      n_runs += s_wt[w];
    }
    n_runs = uni(n_runs);
#pragma unroll
    for (int e = 0; e < kPer; e++)
      if ((hm >> e) & 1u) st[r++] = uint32_t(tid) * kPer + uint32_t(e);
    if (tid == 0) st[n_runs] = W;
    __syncthreads();
    uint64_t sum = 0;
    for (uint32_t q = uint32_t(tid); q < n_runs; q += kSmallThreads) {
      const uint32_t p = st[q], c = st[q + 1] - p;
      sum += c;
      if (b[p] == ra && c == self) s_drop = int32_t(q);
    }
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if (lane == 0 && sum) atomicAdd(&s_sum, (unsigned long long)sum);
    __syncthreads();
    const int32_t drop = uni(s_drop);
    const uint32_t n_keep = n_runs - (drop >= 0 ? 1u : 0u);
    if (tid == 0) {
      s_pos = -1;
      if (s_cur + int64_t(n_keep) > s_end) {
        const int64_t take = max<int64_t>(kSmallSlab, int64_t(n_keep));
        const int64_t nb = int64_t(atomicAdd(A.bump, (unsigned long long)take));
        if (nb + take > A.cap) {
          atomicOr(reinterpret_cast<unsigned long long *>(&A.tot->err), 4ull);
          s_cur = s_end = 0;
        } else {
          s_cur = nb;
          s_end = nb + take;
        }
      }
      if (s_cur + int64_t(n_keep) <= s_end) {
        s_pos = s_cur;
        s_cur += n_keep;
      }
      A.row_base[a] = (n_keep && s_pos >= 0) ? s_pos : 0;
      A.row_nnz[a] = s_pos >= 0 ? int32_t(n_keep) : 0;
      // the row-sum check: the runs (self pairs included) add up to W
      if (s_sum != (unsigned long long)W) {
        atomicOr(reinterpret_cast<unsigned long long *>(&A.tot->err), 2ull);
        A.tot->bad_row = a;
      }
    }
    __syncthreads();
    const int64_t pos = uni(s_pos);
    if (pos >= 0 && SP_CHECK(A, pos + int64_t(n_keep) <= A.cap && n_runs <= W)) {
      for (uint32_t q = uint32_t(tid); q < n_runs; q += kSmallThreads) {
        if (int32_t(q) == drop) continue;
        const uint32_t p = st[q], c = st[q + 1] - p, key = b[p];
        const int64_t o = pos + q - (drop >= 0 && int32_t(q) > drop ? 1 : 0);
        A.col_out[o] = sp_col(A, key);
        A.cnt_out[o] = c - (key == ra ? self : 0u);
      }
    }
    __syncthreads();  // (b and the shared scalars are rewritten by the next row)
  }
}

// ---- tiny rows: one wave per row ------------------------------------------------------------------
// A whole row of at most kTinyW pairs (a streaming window's rows are mostly a few pairs each): its
// contributions' lists are gathered into a per-wave LDS buffer, sorted (bitonic, wave-synchronous),
// equal columns counted (the segmented reduce of the +1 increments), the diagonal's self term removed,
// and the entries written in column order from a per-wave output slab.  No workgroup barrier.
constexpr int kTinyThreads = 256, kTinyWaves = kTinyThreads / 64;
constexpr int64_t kTinySlab = 4096;  // output entries reserved per wave at a time

__device__ inline void tiny_sync() {  // the wave's LDS writes visible to its other lanes
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(kTinyThreads) void k_sp_tiny(SpArgs A) {
  __shared__ uint32_t buf[kTinyWaves][kTinyW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t *b = buf[wave];
  const int64_t first = A.tot->n_chunks - A.tot->n_tiny, n_tiny = A.tot->n_tiny;
  const uint16_t *a0 = reinterpret_cast<const uint16_t *>(A.tarena0);
  const uint32_t *a1 = reinterpret_cast<const uint32_t *>(A.tarena);
  int64_t slab_cur = 0, slab_end = 0;  // (wave-uniform)
  for (;;) {
    int64_t i = 0;
    if (lane == 0) i = int64_t(atomicAdd(reinterpret_cast<unsigned long long *>(&A.tot->tiny_ctr), 1ull));
    i = __shfl(i, 0, 64);
    if (i >= n_tiny) break;
    const SpWork it = A.queue[first + i];
    const int32_t a = it.row;
    const int64_t k0 = it.k0, k1 = it.k1;
    // 1. the contributions' lists (whole lists), 64 at a time, into b in list order
    uint32_t W = 0;
    for (int64_t c0 = k0; c0 < k1; c0 += 64) {
      uint32_t s0 = 0, n0 = 0, s1 = 0, n1 = 0;
      if (c0 + lane < k1) {
        const uint32_t u = A.vals[c0 + lane] & kListMask;
        const int32_t *tbu = A.tb + int64_t(u) * (A.T + 2);
        s0 = uint32_t(tbu[0]);
        n0 = uint32_t(tbu[A.T + 1]) - s0;
        s1 = uint32_t(tbu[1]);
        n1 = uint32_t(tbu[A.T]) - s1;
      }
      const uint32_t len = n0 + n1, inc = wave_incl_scan(len);
      const uint32_t tot = __shfl(inc, 63, 64);
      if (W + tot > uint32_t(kTinyW)) {  // (cannot happen: the planner's W bounds it)
        if (lane == 0) atomicOr(reinterpret_cast<unsigned long long *>(&A.tot->err), 2ull);
        W = 0;
        break;
      }
      uint32_t *d = b + W + inc - len;
      for (uint32_t q = 0; q < n0; q++) d[q] = a0[s0 + q];
      for (uint32_t q = 0; q < n1; q++) d[n0 + q] = a1[s1 + q];
      W += tot;
    }
    // 2. bitonic sort of b[0, n2), padded with kSink
    uint32_t n2 = 1;
    while (n2 < W) n2 <<= 1;
    for (uint32_t q = W + lane; q < n2; q += 64) b[q] = kSink;
    tiny_sync();
    for (uint32_t k = 2; k <= n2; k <<= 1) {
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        for (uint32_t q = lane; q < n2 / 2; q += 64) {
          const uint32_t lo = 2 * q - (q & (j - 1)), hi = lo + j;  // pairs (lo, lo + j) with bit j of lo clear
          const uint32_t x = b[lo], y = b[hi];
          const bool up = (lo & k) == 0;
          if ((x > y) == up) {
            b[lo] = y;
            b[hi] = x;
          }
        }
        tiny_sync();
      }
    }
    // 3. run heads (a 256-bit mask in four ballots), counts, the diagonal's self term
    const uint32_t self = uint32_t(A.spre ? A.spre[k1] - A.spre[k0] : k1 - k0);
    const uint32_t ra = uint32_t(sp_rank(A, a));
    uint64_t hm[kTinyW / 64];
#pragma unroll
    for (int g = 0; g < kTinyW / 64; g++) {
      const uint32_t q = uint32_t(g * 64 + lane);
      const bool h = q < W && (q == 0 || b[q] != b[q - 1]);
      hm[g] = __ballot(h);
    }
    uint32_t my_cnt[kTinyW / 64], n_keep = 0;
    uint64_t keep[kTinyW / 64];
#pragma unroll
    for (int g = 0; g < kTinyW / 64; g++) {
      const uint32_t q = uint32_t(g * 64 + lane);
      uint32_t cnt = 0;
      if ((hm[g] >> lane) & 1ull) {
        uint32_t nx = W;  // the next head after q
        const uint64_t rest = lane < 63 ? hm[g] >> (lane + 1) << (lane + 1) : 0ull;
        if (rest) {
          nx = uint32_t(g * 64 + __ffsll((long long)rest) - 1);
        } else {
#pragma unroll
          for (int g2 = g + 1; g2 < kTinyW / 64; g2++)
            if (nx == W && hm[g2]) nx = uint32_t(g2 * 64 + __ffsll((long long)hm[g2]) - 1);
        }
        cnt = nx - q;
        if (b[q] == ra) cnt -= self;
      }
      my_cnt[g] = cnt;
      keep[g] = __ballot(cnt != 0u);
      n_keep += uint32_t(__popcll(keep[g]));
    }
    // 4. output: the wave's slab; row sum check (counts add up to W - self)
    if (slab_cur + n_keep > slab_end) {
      int64_t nb = 0;
      if (lane == 0) {
        const int64_t take = max<int64_t>(kTinySlab, n_keep);
        nb = int64_t(atomicAdd(A.bump, (unsigned long long)take));
        if (nb + take > A.cap) {
          atomicOr(reinterpret_cast<unsigned long long *>(&A.tot->err), 4ull);
          nb = -1;
        } else {
          nb = nb | (take << 40);  // (take <= 2^23, positions < 2^40)
        }
      }
      nb = __shfl(nb, 0, 64);
      if (nb < 0) break;
      slab_cur = nb & ((int64_t(1) << 40) - 1);
      slab_end = slab_cur + (nb >> 40);
    }
    const int64_t base = slab_cur;
    slab_cur += n_keep;
    uint64_t rsum = 0;
    uint32_t before = 0;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
#pragma unroll
    for (int g = 0; g < kTinyW / 64; g++) {
      if (my_cnt[g]) {
        const int64_t pos = base + before + uint32_t(__popcll(keep[g] & lt));
        A.col_out[pos] = sp_col(A, b[g * 64 + lane]);
        A.cnt_out[pos] = my_cnt[g];
        rsum += my_cnt[g];
      }
      before += uint32_t(__popcll(keep[g]));
    }
    for (int o = 32; o > 0; o >>= 1) rsum += __shfl_xor(rsum, o, 64);
    if (lane == 0) {
      A.row_base[a] = n_keep ? base : 0;
      A.row_nnz[a] = int32_t(n_keep);
      if (rsum != uint64_t(A.rowsum[a])) {
        atomicOr(reinterpret_cast<unsigned long long *>(&A.tot->err), 2ull);
        A.tot->bad_row = a;
      }
    }
    tiny_sync();  // (b is rewritten by the next row)
  }
}

// ---- the hand-written sort path (the default for deferred rows; hipCUB only as the fallback) -------------
// The overflow fallback of the per-row Int2ShortOpenHashMap (ItemRowAggregator.java:21-31) as an MSD radix
// sort by hand: one 1,024-thread workgroup per deferred row.
//  1. the first digit: the row's pairs are partitioned by column tile (kTW columns).  The tile histogram
//     comes from the users' tile tables (tb: a list is already grouped by tile); a wave per contribution
//     reserves its tile segments in the buckets and copies the list with 16-B loads, every id to the
//     bucket of its tile (its high bits) in the row's scratch range; no id is read twice;
//  2. every tile bucket, in column order, becomes (column, count) runs: consecutive buckets of <= kSrbSort
//     ids together are radix-sorted in LDS (block_radix_sort, by the offset in their tile range: two 7-bit
//     passes for one tile) and their runs counted (the segmented reduce of the +1 increments); a larger
//     bucket is counted in kTW LDS counters (a counting sort of the last digit) and compacted in column order.  The
//     runs are written to the front of the row's scratch range (behind the buckets already consumed); the
//     diagonal loses the row's self term (dropped at zero);
//  3. the runs are copied to an exactly sized output slice (relabelled columns mapped back), with the
//     row-sum check of the other paths.
// ~16 B of HBM traffic per pair (segment copy 4 + 4, bucket read 4, run copy) against ~40 for the
// library radix sort of 8-B keys.
constexpr int kSrbThreads = 1024, kSrbWaves = kSrbThreads / 64, kSrbSort = kSmallW;
// buf: sort keys [0, kSrbSort], the other radix buffer from kSrbB, the radix histogram (u16) from kSrbH
constexpr int kSrbB = kSrbSort + 8, kSrbH = kSrbB + kSrbSort + 8, kSrbUsed = kSrbH + (1 << kRadixBits) * kSrbWaves / 2;
static_assert(kSrbUsed <= kTW, "the sort areas share the bucket's LDS counters");

__device__ inline uint32_t srb_block_excl_scan(uint32_t x, uint32_t *total, uint32_t *s_wt) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan(x);
  if (lane == 63) s_wt[wave] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kSrbWaves; w++) {
    const uint32_t v = s_wt[w];
    pre += w < wave ? v : 0u;
    tot += v;
  }
  __syncthreads();
  *total = uni(tot);
  return pre + inc - x;
}

__global__ __launch_bounds__(kSrbThreads) __attribute__((amdgpu_waves_per_eu(8))) void k_srb_row(
    const int32_t *__restrict__ rows, int64_t n_rows, int64_t scr_stride, const int64_t *__restrict__ row_ptr,
    const uint32_t *__restrict__ vals, const int32_t *__restrict__ tb, const uint16_t *__restrict__ arena0,
    const uint32_t *__restrict__ arena1, int32_t T, int32_t Mc, uint32_t *__restrict__ scr_ids,
    uint32_t *__restrict__ scr_cnt, const int64_t *__restrict__ spre, const int64_t *__restrict__ rowsum,
    const int32_t *__restrict__ hot_col, const int32_t *__restrict__ pos_of, int32_t *__restrict__ col_out,
    uint32_t *__restrict__ cnt_out, unsigned long long *__restrict__ bump, int64_t cap,
    int64_t *__restrict__ row_base, int32_t *__restrict__ row_nnz, PlanTotals *__restrict__ tot,
    unsigned long long *__restrict__ srb_st) {
  __shared__ uint32_t buf[kTW];  // dense counters | sorted bucket keys [0, kSrbSort) + run starts above
  __shared__ uint32_t s_hist[kSpMaxTiles + 1], s_off[kSpMaxTiles + 1], s_cur[kSpMaxTiles + 1];
  __shared__ uint32_t s_wt[kSrbWaves];
  __shared__ int32_t s_wdst[kSrbWaves][kSpMaxTiles];  // per wave: a contribution's bucket positions by tile
  __shared__ uint32_t s_o;        // runs written so far (the row's entries)
  __shared__ int32_t s_drop;      // the bucket's run index of a diagonal that drops to zero (-1: none)
  __shared__ unsigned long long s_sum;
  __shared__ int64_t s_base, s_j, s_scur, s_send;  // the row's output base; the dequeued row; the output slab
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // the workgroup's scratch range (every deferred row's pairs fit it); rows dequeued in deferral order
  const int64_t rb = int64_t(blockIdx.x) * scr_stride;
  for (int i = tid; i < kTW; i += kSrbThreads) buf[i] = 0u;
  if (tid == 0) s_scur = s_send = 0;
  bool dirty = false;  // the sort areas of buf hold keys (the counting path needs zero counters)
  for (;;) {
  if (tid == 0) s_j = int64_t(atomicAdd(reinterpret_cast<unsigned long long *>(&tot->srb_ctr), 1ull));
  if (tid <= kSpMaxTiles) {
    s_hist[tid] = 0u;
    s_cur[tid] = 0u;
  }
  if (tid == 0) {
    s_o = 0u;
    s_sum = 0ull;
  }
  __syncthreads();
  const int64_t j = uni(s_j);
  if (j >= n_rows) break;
  const int32_t a = rows[j];
  const uint32_t ra = uint32_t(relabel_pos(pos_of, uint32_t(a)));
  const int64_t k0 = row_ptr[a], k1 = row_ptr[a + 1];
  const uint32_t self = uint32_t(spre ? spre[k1] - spre[k0] : k1 - k0);
  const unsigned long long c_0 = STAT_CLOCK();
  SRB_STAT(5, 1);
  SRB_STAT(6, k1 - k0);
  // 1a. the tile histogram from the tile tables: a wave per contribution, lane t its tile t
  for (int64_t k = k0 + wave; k < k1; k += kSrbWaves) {
    const int32_t *tbu = tb + int64_t(vals[k] & kListMask) * (T + 2);
    if (lane < T) {
      const int32_t n_t = lane == 0 ? tbu[T + 1] - tbu[0] : tbu[lane + 1] - tbu[lane];
      if (n_t > 0) atomicAdd(&s_hist[lane], uint32_t(n_t));
    }
  }
  __syncthreads();
  if (wave == 0) {  // bucket starts: a wave scan of the T <= 64 tile counts
    const uint32_t h = lane < T ? s_hist[lane] : 0u, inc = wave_incl_scan(h);
    if (lane < T) s_off[lane] = inc - h;
    if (lane == T - 1) s_off[T] = inc;
  }
  __syncthreads();
  const unsigned long long c_1 = STAT_CLOCK();
  SRB_STAT(0, c_1 - c_0);
  // 1b. the partition, a wave per contribution: lane t reserves its tile's segment in bucket t; then the
  // wave copies the list with 16-B loads -- the tile-0 part (u16) to bucket 0, the other part (u32, tiles
  // in order) id by id to the bucket of the id's tile (the tile is the id's high bits)
  int32_t *wdst = s_wdst[wave];
  for (int64_t k = k0 + wave; k < k1; k += kSrbWaves) {
    const int32_t *tbu = tb + int64_t(vals[k] & kListMask) * (T + 2);
    const int32_t s0 = tbu[0], n0 = tbu[T + 1] - s0, s1 = tbu[1], n1 = tbu[T] - s1;
    if (lane < T) {
      const int32_t st = lane == 0 ? s0 : tbu[lane];
      const int32_t n_t = lane == 0 ? n0 : tbu[lane + 1] - st;
      const uint32_t d = n_t > 0 ? atomicAdd(&s_cur[lane], uint32_t(n_t)) : 0u;
      // bucket position of the part's position q: wdst[t] + q
      wdst[lane] = int32_t(s_off[lane] + d) - (lane == 0 ? 0 : st - s1);
    }
    tiny_sync();
    const uint4 *p0 = reinterpret_cast<const uint4 *>(arena0 + s0);
    const uint4 *p1 = reinterpret_cast<const uint4 *>(arena1 + s1);
    const uint32_t g0 = (uint32_t(n0) + 7u) >> 3, g1 = (uint32_t(n1) + 3u) >> 2, g = max(g0, g1);
    uint32_t *dst0 = scr_ids + rb + wdst[0];
    for (uint32_t q = uint32_t(lane); q < g; q += 64u) {
      uint4 v0 = make_uint4(0u, 0u, 0u, 0u), v1 = v0;
      if (q < g0) v0 = p0[q];
      if (q < g1) v1 = p1[q];
      if (q < g0) {
        const uint32_t w[4] = {v0.x, v0.y, v0.z, v0.w};
#pragma unroll
        for (int i = 0; i < 8; i++) {
          const uint32_t pos = 8u * q + uint32_t(i);
          if (pos < uint32_t(n0)) dst0[pos] = (w[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
        }
      }
      if (q < g1) {
        const uint32_t w[4] = {v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const uint32_t pos = 4u * q + uint32_t(i);
          if (pos < uint32_t(n1)) scr_ids[rb + wdst[w[i] >> kTShift] + int32_t(pos)] = w[i];
        }
      }
    }
    tiny_sync();  // (wdst is rewritten for the wave's next contribution)
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (the buckets are read back by other waves)
  const unsigned long long c_2 = STAT_CLOCK();
  SRB_STAT(1, c_2 - c_1);
  SRB_STAT(7, s_off[T]);
  // 2. the buckets in column order
  uint64_t sum = 0;
  for (int32_t t = 0; t < T;) {
    const uint32_t n = uni(s_hist[t]);
    if (n == 0) {
      t++;
      continue;
    }
    const uint32_t o = uni(s_o);
    const uint32_t c0 = uint32_t(t) * uint32_t(kTW);
    if (n <= uint32_t(kSrbSort)) {
      // a group: this bucket and the next ones while they fit kSrbSort ids together (contiguous in the
      // scratch), radix-sorted in LDS by their offset in the group's tile range, then its runs
      const unsigned long long c_g = STAT_CLOCK();
      uint32_t g = n;
      int32_t t1 = t + 1;
      while (t1 < T && g + uni(s_hist[t1]) <= uint32_t(kSrbSort)) g += uni(s_hist[t1++]);
      const uint32_t *src = scr_ids + rb + s_off[t];
      uint32_t *ka = buf, *kb = buf + kSrbB;
      {
        static_assert(kSrbSort == 4 * kSrbThreads, "four keys per thread");
        uint32_t v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const uint32_t i = uint32_t(tid) + uint32_t(u) * kSrbThreads;
          v[u] = i < g ? src[i] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const uint32_t i = uint32_t(tid) + uint32_t(u) * kSrbThreads;
          if (i < g) ka[i] = v[u] - c0;
        }
      }
      __syncthreads();
      int bits = kTShift;
      while ((uint32_t(t1 - t) << kTShift) > (1u << bits)) bits++;
      const uint32_t *ks = block_radix_sort<kSrbThreads>(ka, kb, reinterpret_cast<uint16_t *>(buf + kSrbH), s_wt, g,
                                                         bits);
      uint32_t *st = ks == ka ? kb : ka;  // run starts in the free area (+1: the end marker)
      dirty = true;
      uint32_t hm = 0;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const uint32_t i = 4u * uint32_t(tid) + uint32_t(e);
        if (i < g && (i == 0 || ks[i] != ks[i - 1])) hm |= 1u << e;
      }
      uint32_t n_runs;
      const uint32_t r0 = srb_block_excl_scan(uint32_t(__popc(hm)), &n_runs, s_wt);
      if (tid == 0) s_drop = -1;
      {
        uint32_t r = r0;
#pragma unroll
        for (int e = 0; e < 4; e++)
          if ((hm >> e) & 1u) st[r++] = 4u * uint32_t(tid) + uint32_t(e);
      }
      if (tid == 0) st[n_runs] = g;
      __syncthreads();
      for (uint32_t r = tid; r < n_runs; r += kSrbThreads) {
        const uint32_t p = st[r], c = st[r + 1] - p;
        sum += c;
        if (ks[p] + c0 == ra && c == self) s_drop = int32_t(r);
      }
      __syncthreads();
      const int32_t drop = uni(s_drop);
      for (uint32_t r = tid; r < n_runs; r += kSrbThreads) {
        if (int32_t(r) == drop) continue;
        const uint32_t p = st[r], c = st[r + 1] - p, col = ks[p] + c0;
        const uint32_t q = o + r - (drop >= 0 && int32_t(r) > drop ? 1u : 0u);
        scr_ids[rb + q] = col;
        scr_cnt[rb + q] = c - (col == ra ? self : 0u);
      }
      if (tid == 0) s_o = o + n_runs - (drop >= 0 ? 1u : 0u);
      __syncthreads();
      SRB_STAT(2, STAT_CLOCK() - c_g);
      SRB_STAT(8, 1);
      t = t1;
    } else {
      // counting sort of the bucket's last digit: kTW LDS counters, then a column-order compaction
      const unsigned long long c_c = STAT_CLOCK();
      if (dirty) {
        for (uint32_t i = tid; i < uint32_t(kSrbUsed); i += kSrbThreads) buf[i] = 0u;
        dirty = false;
        __syncthreads();
      }
      const uint32_t *src = scr_ids + rb + s_off[t];
      const uint32_t w = uint32_t(min(int64_t(kTW), int64_t(Mc) - int64_t(c0)));
      for (uint32_t i0 = 0; i0 < n; i0 += 8u * kSrbThreads) {  // (8 loads in flight per thread)
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const uint32_t i = i0 + uint32_t(tid) + uint32_t(u) * kSrbThreads;
          v[u] = i < n ? src[i] : kSink;
        }
#pragma unroll
        for (int u = 0; u < 8; u++)
          if (v[u] != kSink) atomicAdd(&buf[v[u] - c0], 1u);
      }
      __syncthreads();
      if (tid == 0 && ra >= c0 && ra < c0 + w) buf[ra - c0] -= self;  // (the self pairs were counted too)
      __syncthreads();
      constexpr uint32_t per = uint32_t(kTW) / kSrbWaves;  // columns per wave (1,024)
      const uint32_t lo = min(w, uint32_t(wave) * per), hi = min(w, lo + per);
      uint32_t c = 0;
      for (uint32_t b = lo + lane; b < hi; b += 64) c += buf[b] != 0u;
      for (int x = 32; x > 0; x >>= 1) c += __shfl_xor(c, x, 64);
      uint32_t n_out;
      uint32_t off = srb_block_excl_scan(lane == 0 ? c : 0u, &n_out, s_wt);
      off = __shfl(off, 0, 64);
      const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
      for (uint32_t b0 = lo; b0 < hi; b0 += 64) {
        const uint32_t b = b0 + uint32_t(lane);
        const uint32_t v = b < hi ? buf[b] : 0u;
        const uint64_t m = __ballot(v != 0u);
        if (v) {
          const uint32_t q = o + off + uint32_t(__popcll(m & lt));
          scr_ids[rb + q] = c0 + b;
          scr_cnt[rb + q] = v;
          sum += v;
          buf[b] = 0u;
        }
        off += uint32_t(__popcll(m));
      }
      if (tid == 0) {
        s_o = o + n_out;
        if (ra >= c0 && ra < c0 + w) sum += self;  // (sum counts the self pairs on both paths)
      }
      __syncthreads();
      SRB_STAT(3, STAT_CLOCK() - c_c);
      SRB_STAT(9, 1);
      t++;
    }
  }
  const unsigned long long c_3 = STAT_CLOCK();
  // 3. the exact output slice; the row-sum check
  for (int x = 32; x > 0; x >>= 1) sum += __shfl_xor(sum, x, 64);
  if (lane == 0 && sum) atomicAdd(&s_sum, (unsigned long long)sum);
  __syncthreads();
  const uint32_t d = s_o;
  if (tid == 0) {
    // the row's slice from the workgroup's output slab (a new slab of >= kSmallSlab entries when it is short)
    int64_t b = -1;
    if (s_scur + int64_t(d) > s_send) {
      const int64_t take = max<int64_t>(kSmallSlab, int64_t(d));
      const int64_t nb = int64_t(atomicAdd(bump, (unsigned long long)take));
      if (nb + take > cap) {
        atomicOr(reinterpret_cast<unsigned long long *>(&tot->err), 4ull);
        s_scur = s_send = 0;
      } else {
        s_scur = nb;
        s_send = nb + take;
      }
    }
    if (s_scur + int64_t(d) <= s_send) {
      b = s_scur;
      s_scur += d;
    }
    s_base = b;
    row_base[a] = (b < 0 || d == 0) ? 0 : b;
    row_nnz[a] = b < 0 ? 0 : int32_t(d);
    if (s_sum != (unsigned long long)(rowsum[a] + self)) {
      atomicOr(reinterpret_cast<unsigned long long *>(&tot->err), 2ull);
      tot->bad_row = a;
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const int64_t base = s_base;
  (void)c_3;
  for (uint32_t i0 = 0; base >= 0 && i0 < d; i0 += 4u * kSrbThreads) {  // (4 entries' loads in flight per thread)
    uint32_t c[4], n[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t i = i0 + uint32_t(tid) + uint32_t(u) * kSrbThreads;
      c[u] = i < d ? scr_ids[rb + i] : 0u;
      n[u] = i < d ? scr_cnt[rb + i] : 0u;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t i = i0 + uint32_t(tid) + uint32_t(u) * kSrbThreads;
      if (i < d) {
        col_out[base + i] = relabel_col(hot_col, c[u]);
        cnt_out[base + i] = n[u];
      }
    }
  }
  SRB_STAT(4, STAT_CLOCK() - c_3);
  SRB_STAT(10, STAT_CLOCK() - c_0);
  __builtin_amdgcn_s_waitcnt(0);  // (the next row's partition rewrites the scratch these loads read)
  __syncthreads();
  }
}

__global__ void k_sr_pair_work(const int32_t *__restrict__ rows, int64_t n, const int64_t *__restrict__ row_w,
                               int64_t *__restrict__ out) {
  const int64_t j = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j < n) out[j] = row_w[rows[j]];
}

inline unsigned nblocks(int64_t n, int t) { return unsigned((n + t - 1) / t); }

int bits_for(int64_t v) {
  int b = 1;
  while ((int64_t(1) << b) < v) b++;
  return b;
}

}  // namespace

namespace {

// Item frequencies of a log (the multi-GPU owner map and the planner's column estimate).  Zipf logs put most
// interactions on a few items, whose global counters would serialise at L2 under per-interaction atomics;
// each workgroup therefore keeps the items it sees most in an LDS table (open addressing: an item claims a
// slot with a compare-and-swap, kHistProbe probes at most) and flushes it once; an item that finds no slot
// (the table is full of the workgroup's earlier items) goes to a global 64-bit atomic -- such items are rare
// in the workgroup's share, so their counters are not contended.  Whatever order the ids come in.
constexpr int kHistSlots = 8192, kHistProbe = 8, kHistThreads = 1024;
__global__ __launch_bounds__(kHistThreads) void k_item_counts(const int32_t *__restrict__ items, int64_t n, int32_t M,
                                                              unsigned long long *__restrict__ counts) {
  __shared__ uint32_t hk[kHistSlots], hc[kHistSlots];
  for (int i = threadIdx.x; i < kHistSlots; i += kHistThreads) {
    hk[i] = 0u;
    hc[i] = 0u;
  }
  __syncthreads();
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;  // a contiguous share per workgroup
  const int64_t i0 = int64_t(blockIdx.x) * per, i1 = min(n, i0 + per);
  for (int64_t i = i0 + threadIdx.x; i < i1; i += kHistThreads) {
    const uint32_t it = uint32_t(items[i]);
    if (it >= uint32_t(M)) continue;
    const uint32_t key = it + 1u;
    uint32_t h = (it * 0x9E3779B1u) >> (32 - 13);
    bool done = false;
    for (int p = 0; p < kHistProbe; p++) {
      const uint32_t cur = atomicCAS(hk + h, 0u, key);
      if (cur == 0u || cur == key) {
        atomicAdd(hc + h, 1u);
        done = true;
        break;
      }
      h = (h + 1u) & (kHistSlots - 1u);
    }
    if (!done) atomicAdd(counts + it, 1ull);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kHistSlots; i += kHistThreads)
    if (hk[i]) atomicAdd(counts + (hk[i] - 1u), (unsigned long long)hc[i]);
}
}  // namespace

Status launch_item_counts(hipStream_t s, const int32_t *items, int64_t n, int32_t M, int64_t *counts) {
  COOC_HIP_TRY(hipMemsetAsync(counts, 0, sizeof(int64_t) * size_t(M), s));
  if (n > 0) {
    int dev = 0, n_cu = 256;
    COOC_HIP_TRY(hipGetDevice(&dev));
    COOC_HIP_TRY(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    const int64_t want = (n + 4095) / 4096;
    k_item_counts<<<unsigned(std::max<int64_t>(1, std::min<int64_t>(want, int64_t(n_cu) * 2))), kHistThreads, 0, s>>>(
        items, n, M, reinterpret_cast<unsigned long long *>(counts));
    COOC_HIP_TRY(hipGetLastError());
  }
  return Status::Ok();
}

Status Counter::run_sparse(int64_t U, const int64_t *up, const int32_t *items, int64_t n, hipStream_t s,
                           CountResult *out, KernelTimer *timer, const int32_t *owner, int32_t part,
                           const int64_t *freq, int64_t n_freq, const SparseWindow *win) {
  const int32_t M = M_;
  // 0. column relabel (batch windows; not streaming ones, whose delta rows merge into column-ordered global
  // rows): the batch's kTW most frequent items -- its own frequencies, or the caller's global counts -- become
  // tile 0 and the rest move one tile up (k_relabel_*), so that the hot columns fill the u16 tile 0 and the
  // tiling works whatever order the ids come in.  Rows come out in that column order (CountResult.rank_of).
  // Mc: the columns of the relabelled space (M + kTW; holes where the hot items were).
  // (the relabel is dropped again below when the ids already put the hot items in tile 0)
  bool relabel = relabel_ && !win && M > kTW && int64_t(M) + kTW <= int64_t(kSpMaxTiles) * kTW;
  int32_t Mc = relabel ? M + kTW : M;
  int32_t T = int32_t((int64_t(Mc) + kTW - 1) / kTW);
  if (T > kSpMaxTiles)
    return Status{1, "n_items > " + std::to_string(int64_t(kSpMaxTiles) * kTW) + " is not supported"};
  if (n > int64_t(INT32_MAX)) return Status{1, "more than 2^31 interactions in one window"};
  // (a contribution keeps its list index in bits 0..30, kSelfBit in bit 31)
  if (U > int64_t(kListMask)) return Status{1, "more than 2^31 - 1 user lists in one window"};
  const int64_t U1 = std::max<int64_t>(U, 1), n1 = std::max<int64_t>(n, 1);
  COOC_TRY(tot_.reserve(sizeof(PlanTotals)));
  COOC_TRY(queue_.reserve(sizeof(int32_t) * 4));
  COOC_TRY(keys_in_.reserve(sizeof(uint32_t) * (n1 + 1)));
  COOC_TRY(vals_in_.reserve(sizeof(uint32_t) * (n1 + 1)));
  COOC_TRY(keys_out_.reserve(sizeof(uint32_t) * (n1 + 1)));
  COOC_TRY(vals_out_.reserve(sizeof(uint32_t) * (n1 + 1)));
  const int64_t n_groups0 = (n1 + 7 * U1) / 8 + 4, n_groups1 = (n1 + 3 * U1) / 4 + 4;
  COOC_TRY(sp_arena_.reserve(sizeof(uint4) * size_t(n_groups1)));   // arena1: lists padded to 4 ids
  COOC_TRY(sp_arena0_.reserve(sizeof(uint4) * size_t(n_groups0)));  // arena0: tile-0 ids padded to 8
  COOC_TRY(sp_pbase_.reserve(sizeof(uint64_t) * size_t(2 * U1 + 1)));  // packed region lengths, their prefix
  COOC_TRY(sp_ulen_.reserve(sizeof(uint32_t) * size_t(U1)));  // list lengths (u32) for the pair-work prefix
  COOC_TRY(sp_tb_.reserve(sizeof(int32_t) * size_t(U1) * size_t(T + 2)));
  if (8 * n_groups0 > int64_t(INT32_MAX)) return Status{1, "more than 2^31 arena positions in one window"};
  COOC_TRY(epre_.reserve(sizeof(int64_t) * (n1 + 1)));
  COOC_TRY(row_ptr_.reserve(sizeof(int64_t) * (M + 1)));
  COOC_TRY(rowsum_.reserve(sizeof(int64_t) * M));
  COOC_TRY(row_base_.reserve(sizeof(int64_t) * (M + 1)));
  COOC_TRY(row_nnz_.reserve(sizeof(int32_t) * M));
  COOC_TRY(sp_roww_.reserve(sizeof(int64_t) * M));
  COOC_TRY(sp_pstart_.reserve(sizeof(uint64_t) * M));
  COOC_TRY(sp_pdense_.reserve(sizeof(uint64_t) * M));
  COOC_TRY(sp_hz_.reserve(sizeof(uint64_t) * 2 * M));
  COOC_TRY(order_keys_.reserve(sizeof(uint64_t) * 2 * M));
  COOC_TRY(order_.reserve(sizeof(int32_t) * 2 * M));
  COOC_TRY(row_nch_.reserve(sizeof(int32_t) * M));           // work items per row (split rows)
  COOC_TRY(ord_nch_.reserve(sizeof(int32_t) * M));           // ... in sorted order
  COOC_TRY(ord_cbase_.reserve(sizeof(int32_t) * (M + 1)));   // ... exclusive prefix
  COOC_TRY(sp_est_.reserve(sizeof(float) * (T * kEstK + T)));
  PlanTotals *tot = tot_.as<PlanTotals>();
  uint32_t *keys_in = keys_in_.as<uint32_t>(), *vals_in = vals_in_.as<uint32_t>();
  uint32_t *keys = keys_out_.as<uint32_t>(), *vals = vals_out_.as<uint32_t>();
  int64_t *epre = epre_.as<int64_t>(), *row_ptr = row_ptr_.as<int64_t>();
  float *est = sp_est_.as<float>(), *gmass = est + T * kEstK;  // (gmass moves if T shrinks below)
  int32_t *qctr = queue_.as<int32_t>();
  COOC_HIP_TRY(hipMemsetAsync(tot, 0, sizeof(PlanTotals), s));
  COOC_HIP_TRY(hipMemsetAsync(epre, 0, sizeof(int64_t), s));

  // the planner's sorts and its select: hand-written (cooc_radix.h) unless COOC_LIB_SORTS=1 (the hipCUB calls,
  // an A/B knob)
  static const bool lib_sorts = [] {
    const char *e = getenv("COOC_LIB_SORTS");
    return e && e[0] == '1';
  }();
  const int kb = bits_for(M);
  size_t tmp = 0, q = 0;
  if (lib_sorts) {
    COOC_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, q, keys_in, keys, vals_in, vals, int(n1), 0, kb, s));
    tmp = std::max(tmp, q);
    COOC_HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, q, order_keys_.as<uint64_t>(),
                                                              order_keys_.as<uint64_t>() + M, order_.as<int32_t>(),
                                                              order_.as<int32_t>() + M, M, 0, 64, s));
    tmp = std::max(tmp, q);
  } else {
    tmp = std::max({radix_sort_tmp_bytes<uint32_t, uint32_t>(n1), radix_sort_tmp_bytes<uint64_t, int32_t>(M),
                    select_tmp_bytes(M)});
  }
  uint64_t *plen = sp_pbase_.as<uint64_t>(), *pbase = plen + U1;
  COOC_TRY(sort_tmp_.reserve(tmp));
  // the planner's prefix sums (cooc_scan.h): tile statuses for the largest of them, reserved once up front
  COOC_TRY(scan_state_.reserve(sizeof(unsigned long long) *
                               size_t(scan_state_words(std::max({n1, U1, int64_t(M), win ? win->n_contrib : int64_t(0)})))));
  unsigned long long *scan_st = scan_state_.as<unsigned long long>();
  int64_t *scan_err = &tot->err;
  uint32_t *ulen = sp_ulen_.as<uint32_t>();
  if (U > 0) k_list_len32<<<nblocks(U, 256), 256, 0, s>>>(U, up, ulen);

  const int64_t waves = std::min<int64_t>(std::max<int64_t>(U, 1), 65536);
  int32_t *hot_col = nullptr, *pos_of = nullptr;
  const uint8_t *hot_u8 = nullptr;    // 1 per hot id (tile 0 after the relabel)
  const int64_t *freq_col = nullptr;  // the frequencies in relabelled column order (the planner's estimate)
  bool sorted_early = false;          // contributions sorted ahead of the relabel (no owner)
  if (relabel) {
    COOC_TRY(sp_rank_.reserve(sizeof(int32_t) * size_t(3 * M + kTW + 8) + size_t(M)));
    COOC_TRY(sp_rkeys_.reserve(sizeof(uint64_t) * size_t(2 * M) + sizeof(int64_t) * size_t(Mc)));
    pos_of = sp_rank_.as<int32_t>();
    hot_col = pos_of + M;
    int32_t *ids = hot_col + kTW, *order = ids + M, *n_sel = order + M;
    uint8_t *hot = reinterpret_cast<uint8_t *>(n_sel + 8);
    uint64_t *rk_in = sp_rkeys_.as<uint64_t>(), *rk_out = rk_in + M;
    int64_t *fc = reinterpret_cast<int64_t *>(rk_out + M);
    int64_t n_tot = n;
    if (!owner) {  // the log's own frequencies: the row lengths of the item-sorted contributions
      if (U > 0) k_sp_contribs<<<nblocks(waves * 64, 256), 256, 0, s>>>(U, up, items, M, keys_in, vals_in);
      if (n > 0) {
        size_t b = sort_tmp_.cap;
        if (lib_sorts)
          COOC_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(sort_tmp_.p, b, keys_in, keys, vals_in, vals, int(n), 0, kb, s));
        else
          COOC_TRY(radix_sort_pairs(keys_in, vals_in, keys, vals, n, 0, kb, false, sort_tmp_.p, s));
        COOC_TRY(launch_scan<true>(ScanUserLen{vals, ulen}, epre + 1, n, scan_st, scan_err, s));
      }
      k_sp_row_ptr<<<nblocks(int64_t(M) + 1, 256), 256, 0, s>>>(keys, n, M, row_ptr);
      sorted_early = true;
    } else {
      n_tot = n_freq;
    }
    k_rank_keys<<<nblocks(M, 256), 256, 0, s>>>(row_ptr, owner ? freq : nullptr, M, rk_in, ids, hot);
    size_t b = 0, b2 = 0;
    const int fb = bits_for(std::max<int64_t>(n_tot, 1) + 1);
    hipcub::CountingInputIterator<int32_t> from0(0);
    if (lib_sorts) {
      COOC_HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, b, rk_in, rk_out, ids, order, M, 0, fb, s));
      COOC_HIP_TRY(hipcub::DeviceSelect::If(nullptr, b2, from0, hot_col, n_sel, M, IsHot{hot}, s));
    }
    COOC_TRY(sort_tmp_.reserve(std::max({b, b2, tmp})));
    b = sort_tmp_.cap;
    if (lib_sorts)
      COOC_HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(sort_tmp_.p, b, rk_in, rk_out, ids, order, M, 0, fb, s));
    else
      COOC_TRY(radix_sort_pairs(rk_in, ids, rk_out, order, M, 0, fb, true, sort_tmp_.p, s));
    k_hot_mark<<<nblocks(kTW, 256), 256, 0, s>>>(order, kTW, hot);
    b = sort_tmp_.cap;
    if (lib_sorts)
      COOC_HIP_TRY(hipcub::DeviceSelect::If(sort_tmp_.p, b, from0, hot_col, n_sel, M, IsHot{hot}, s));  // kTW of them
    else
      COOC_TRY(select_flagged(hot, M, hot_col, n_sel, sort_tmp_.p, s));
    // ids that already put (nearly) every hot item in tile 0 keep their order: the relabel would only add
    // its lookups (an item-ranked log; measured 4 ms per C3 share)
    {
      int32_t *d_ov = n_sel + 4;
      COOC_HIP_TRY(hipMemsetAsync(d_ov, 0, sizeof(int32_t), s));
      k_hot_overlap<<<nblocks(kTW, 256), 256, 0, s>>>(hot, kTW, d_ov);
      int32_t ov = 0;
      COOC_HIP_TRY(hipMemcpyAsync(&ov, d_ov, sizeof(int32_t), hipMemcpyDeviceToHost, s));
      COOC_HIP_TRY(hipStreamSynchronize(s));
      last_hot_overlap_ = ov;
#ifdef COOC_SP_STATS
      fprintf(stderr, "[sp] relabel: %d of the %d hot items have ids below %d -> %s\n", ov, kTW, kTW,
              ov >= kTW - kTW / 16 ? "kept ids" : "relabelled");
#endif
      if (ov >= kTW - kTW / 16) {
        relabel = false;
        Mc = M;
        T = int32_t((int64_t(Mc) + kTW - 1) / kTW);
        gmass = est + T * kEstK;
        pos_of = hot_col = nullptr;
      }
    }
    if (relabel) {
      k_relabel_pos<<<nblocks(M, 256), 256, 0, s>>>(hot, rk_in, M, pos_of, fc);
      hot_u8 = hot;
      k_relabel_hot<<<nblocks(kTW, 256), 256, 0, s>>>(hot_col, rk_in, pos_of, fc);
      COOC_HIP_TRY(hipGetLastError());
      freq_col = fc;
    }
  }
  last_hot_col_ = hot_col;
  last_pos_of_ = pos_of;
  last_mc_ = Mc;
  // the bitmaps of the user passes (hot ids after a relabel; the part's rows)
  const int64_t n_words = (int64_t(M) + 31) / 32;
  COOC_TRY(sp_bits_.reserve(sizeof(uint32_t) * size_t(2 * n_words + 2)));
  uint32_t *hotbm = relabel ? sp_bits_.as<uint32_t>() : nullptr;
  uint32_t *minebm = owner ? sp_bits_.as<uint32_t>() + n_words : nullptr;
  if (hotbm) k_bits_hot<<<nblocks(n_words, 256), 256, 0, s>>>(hot_u8, M, hotbm);
  if (minebm) k_bits_owner<<<nblocks(n_words, 256), 256, 0, s>>>(owner, part, M, minebm);
  // 1. per-user tile regrouping + the (item, user) contributions (owner != NULL: of this part's rows)
  if (owner) {
    COOC_TRY(sp_ownc_.reserve(sizeof(int32_t) * size_t(U1)));
    COOC_TRY(sp_ownoff_.reserve(sizeof(int64_t) * size_t(U1 + 1)));
  }
  COOC_HIP_TRY(hipMemsetAsync(pbase, 0, sizeof(uint64_t), s));
  if (U > 0) {
    k_sp_tile_counts<<<nblocks(waves * 64, 256), 256, 0, s>>>(U, up, items, M, plen, owner, part,
                                                             sp_ownc_.as<int32_t>(), pos_of, hotbm, minebm);
    COOC_TRY(launch_scan<true>(ScanU64{plen}, pbase + 1, U, scan_st, scan_err, s));
  }
  int64_t *ownoff = owner ? sp_ownoff_.as<int64_t>() : nullptr;
  if (owner) {  // owned contributions per user -> their offsets
    COOC_HIP_TRY(hipMemsetAsync(ownoff, 0, sizeof(int64_t), s));
    if (U > 0) {
      COOC_TRY(launch_scan<true>(ScanI32{sp_ownc_.as<int32_t>()}, ownoff + 1, U, scan_st, scan_err, s));
    }
  }
  if (U > 0) {
    k_sp_tile_lists<<<nblocks(waves * 64, 256), 256, 0, s>>>(U, up, items, M, T, sp_tb_.as<int32_t>(),
                                                            sp_arena0_.as<uint16_t>(), sp_arena_.as<uint32_t>(), pbase,
                                                            (win || sorted_early) ? nullptr : keys_in, vals_in, owner,
                                                            part, ownoff, tot, pos_of, hotbm, minebm);
    COOC_HIP_TRY(hipGetLastError());
  }
  int64_t n_c = n;  // contributions: every interaction, or those of the owned rows, or a window's positions
  if (win) {
    n_c = win->n_contrib;
    if (win->n_users > 0)
      k_sp_window_contribs<<<nblocks(std::min<int64_t>(win->n_users, 65536) * 64, 256), 256, 0, s>>>(
          win->n_users, up, items, win->old, win->cbase, keys_in, vals_in);
    COOC_HIP_TRY(hipGetLastError());
  }
  if (owner) {
    COOC_HIP_TRY(hipMemcpyAsync(&n_c, ownoff + U, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    COOC_HIP_TRY(hipStreamSynchronize(s));
  }
  SPT("partition");
  // 2. regroup by row (the keyBy(itemA) of FlinkCooccurrences.java:152); 3. row pointer; 4. pair work
  if (n_c > 0 && !sorted_early) {
    size_t b = sort_tmp_.cap;
    if (lib_sorts)
      COOC_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(sort_tmp_.p, b, keys_in, keys, vals_in, vals, int(n_c), 0, kb, s));
    else
      COOC_TRY(radix_sort_pairs(keys_in, vals_in, keys, vals, n_c, 0, kb, false, sort_tmp_.p, s));
    COOC_TRY(launch_scan<true>(ScanUserLen{vals, ulen}, epre + 1, n_c, scan_st, scan_err, s));
  }
  int64_t *spre = nullptr;  // a window's self flags, prefix in row order
  if (win) {
    COOC_TRY(sp_spre_.reserve(sizeof(int64_t) * size_t(n_c + 2)));
    spre = sp_spre_.as<int64_t>();
    COOC_HIP_TRY(hipMemsetAsync(spre, 0, sizeof(int64_t), s));
    if (n_c > 0) {
      COOC_TRY(launch_scan<true>(ScanSelfFlag{vals}, spre + 1, n_c, scan_st, scan_err, s));
    }
  }
  SPT("sort+scan");
  if (!sorted_early) k_sp_row_ptr<<<nblocks(int64_t(M) + 1, 256), 256, 0, s>>>(keys, n_c, M, row_ptr);
  // 5. expected distinct keys per tile; 6. per-row plan
  // column frequencies: of this log's interactions (owner == NULL), else the caller's global counts; in rank
  // order after a relabel
  const int64_t n_est = freq ? n_freq : win ? n_c : n;
  if (n_est > 0) k_sp_est<<<dim3(T, kEstK), 256, 0, s>>>(row_ptr, relabel ? freq_col : freq, Mc, n_est, est, gmass);
  else COOC_HIP_TRY(hipMemsetAsync(est, 0, sizeof(float) * (T * kEstK + T), s));
  SPT("est");
  k_sp_plan<<<nblocks(M, 256), 256, 0, s>>>(M, T, row_ptr, epre, est, gmass, rowsum_.as<int64_t>(),
                                            sp_roww_.as<int64_t>(), sp_pstart_.as<uint64_t>(),
                                            sp_pdense_.as<uint64_t>(), sp_hz_.as<uint64_t>(),
                                            order_keys_.as<uint64_t>(),
                                            order_.as<int32_t>(), row_nch_.as<int32_t>(), row_nnz_.as<int32_t>(),
                                            row_base_.as<int64_t>(), tot, spre, (small_off_ ? 1 : 3) | (mid_off_ ? 0 : 4));
  k_sp_totals<<<1, 1, 0, s>>>(tot, epre, spre, n_c, qctr);  // n_chunks is recomputed below once n_split is final
  COOC_HIP_TRY(hipGetLastError());
  COOC_HIP_TRY(hipMemcpyAsync(h_tot_, tot, sizeof(PlanTotals), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  if (h_tot_->err & 1) return Status{1, "item id outside [0, n_items)"};
  if (h_tot_->err & 8) return Status{2, "internal bounds check failed (planner prefix sum)"};
  const int64_t n_split = h_tot_->n_split;
  const int64_t n_work = h_tot_->n_chunks;
  const int64_t work_total = h_tot_->work_total, self_total = h_tot_->self_total;
  const int64_t bound = h_tot_->cap_total, est_nnz = h_tot_->est_nnz;

  SPT("plan+sync");
#ifdef COOC_SP_TRACE
  {
    std::vector<uint64_t> ps(M), pd(M);
    std::vector<int64_t> rw(M);
    std::vector<float> es(T * kEstK + T);
    hipMemcpy(ps.data(), sp_pstart_.p, 8 * M, hipMemcpyDeviceToHost);
    hipMemcpy(pd.data(), sp_pdense_.p, 8 * M, hipMemcpyDeviceToHost);
    hipMemcpy(rw.data(), sp_roww_.p, 8 * M, hipMemcpyDeviceToHost);
    hipMemcpy(es.data(), est, 4 * (T * kEstK + T), hipMemcpyDeviceToHost);
    for (int t = 0; t < T; t++) fprintf(stderr, "[sp] tile %d gmass %g est[0] %g est[20] %g est[40] %g\n", t, es[T * kEstK + t], es[t * kEstK], es[t * kEstK + 20], es[t * kEstK + 40]);
    int shown = 0;
    for (int a = 0; a < M && shown < 12; a++)
      if (rw[a] > 0) { fprintf(stderr, "[sp] row %d W %lld start %llx dense %llx\n", a, (long long)rw[a], (unsigned long long)ps[a], (unsigned long long)pd[a]); shown++; }
  }
#endif
  // 7. work queue: rows by pair work (descending); split rows' work items first
  COOC_TRY(sp_queue_.reserve(sizeof(SpWork) * size_t(std::max<int64_t>(n_work, 1))));
  COOC_TRY(split_row_.reserve(sizeof(int32_t) * std::max<int64_t>(n_split, 1)));
  COOC_TRY(split_slot_.reserve(sizeof(int32_t) * M));
  {
    // the keys are the rows' pair work, at most work_total: only its bits are sorted (C3's 1/8 share: 35 of 64,
    // five 8-bit passes instead of eight; the same order)
    size_t b = sort_tmp_.cap;
    const int wb = std::min(64, bits_for(work_total + 1));
    if (lib_sorts)
      COOC_HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(sort_tmp_.p, b, order_keys_.as<uint64_t>(),
                                                                order_keys_.as<uint64_t>() + M, order_.as<int32_t>(),
                                                                order_.as<int32_t>() + M, M, 0, wb, s));
    else
      COOC_TRY(radix_sort_pairs(order_keys_.as<uint64_t>(), order_.as<int32_t>(), order_keys_.as<uint64_t>() + M,
                                order_.as<int32_t>() + M, M, 0, wb, true, sort_tmp_.p, s));
    k_sp_gather_nwork<<<nblocks(M, 256), 256, 0, s>>>(order_.as<int32_t>() + M, row_nch_.as<int32_t>(), M,
                                                      ord_nch_.as<int32_t>());
    COOC_TRY(launch_scan<false>(ScanI32{ord_nch_.as<int32_t>()}, ord_cbase_.as<int32_t>(), M, scan_st, scan_err, s));
    k_sp_queue<<<nblocks(M, 256), 256, 0, s>>>(order_.as<int32_t>() + M, order_keys_.as<uint64_t>() + M,
                                              ord_cbase_.as<int32_t>(), gmass, row_ptr, sp_pstart_.as<uint64_t>(),
                                              sp_pdense_.as<uint64_t>(), sp_hz_.as<uint64_t>(), M, T, tot,
                                              sp_queue_.as<SpWork>(),
                                              split_slot_.as<int32_t>(), split_row_.as<int32_t>(),
                                              row_nnz_.as<int32_t>());
    COOC_HIP_TRY(hipGetLastError());
  }
  SPT("queue");
  const int64_t sstride = (int64_t(Mc) + 3) & ~int64_t(3);  // 16-B aligned staging rows (relabelled columns)
  if (n_split > 0) {
    const size_t need = sizeof(uint32_t) * size_t(n_split) * size_t(sstride);
    COOC_TRY(staging_.reserve(need));
  }
  // gather scratch: a bucket region per workgroup for the largest expected tail (+25%); a work item
  // whose exact tail is larger walks per chunk instead.  Skipped when memory is short.
  // the two shapes' launches: the queue's big rows and split shares [0, n_big), then its mid rows
  const int64_t n_tiny = h_tot_->n_tiny, n_small = h_tot_->n_small, n_mid = h_tot_->n_mid;
  const int64_t n_big = n_work - n_tiny - n_small - n_mid;
  COOC_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(k_sp_main<SpBig>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, SpBig::kLds));
  COOC_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(k_sp_main<SpMid>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, SpMid::kLds));
  int per_cu = 1, per_cu_mid = 1;
  COOC_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sp_main<SpBig>, SpBig::kThreads, SpBig::kLds));
  COOC_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_mid, k_sp_main<SpMid>, SpMid::kThreads, SpMid::kLds));
  const int64_t grid = std::min<int64_t>(std::max<int64_t>(n_big, 1), int64_t(n_cu_) * std::max(1, per_cu));
  const int64_t grid_mid = std::min<int64_t>(std::max<int64_t>(n_mid, 1), int64_t(n_cu_) * std::max(1, per_cu_mid));
  last_mid_grid_ = n_mid > 0 ? grid_mid : 0;
  // gather scratch (per launch): a bucket region per workgroup for the largest expected tail (+25%); a work item
  // whose exact tail is larger walks per chunk instead.  Skipped when memory is short.
  auto scratch = [&](int64_t max_tail, int64_t g, DevBuf &buf) -> int64_t {
    if (max_tail <= 0) return 0;
    const int64_t sc = std::min<int64_t>(kScrGroups, (max_tail + max_tail / 4 + 64 * T + 4096) / 4 + 1);
    const size_t need = sizeof(uint4) * size_t(g) * size_t(sc);
    size_t f0 = 0, t0 = 0;
    if (hipMemGetInfo(&f0, &t0) != hipSuccess) return 0;
    if (need > buf.cap && (need > (f0 + buf.cap) / 4 || !buf.reserve(need).ok())) return 0;
    return sc;
  };
  const int64_t scr_cap = scratch(h_tot_->max_tail, grid, sp_scr_);
  const int64_t scr_cap_mid = n_mid > 0 ? scratch(h_tot_->max_tail_mid, grid_mid, sp_scr_mid_) : 0;
  const int64_t n_gather = h_tot_->n_gather_rows + h_tot_->n_split_work;  // gather items (bound)
  // 8. output region: the expected entries plus slab slack, at most the exact bound
  size_t free_b = 0, total_b = 0;
  COOC_HIP_TRY(hipMemGetInfo(&free_b, &total_b));
  const int64_t slab = std::max<int64_t>(int64_t(1) << 16, std::min<int64_t>(int64_t(1) << 22, est_nnz / (8 * grid)));
  const int64_t grid_tiny = std::min<int64_t>((n_tiny + kTinyWaves - 1) / kTinyWaves, int64_t(n_cu_) * 8);
  const int64_t grid_small = std::min<int64_t>(n_small, int64_t(n_cu_) * 4);
  const int64_t slack = 2 * grid * slab + (n_mid ? 2 * grid_mid * slab : 0) + M +
                        (n_tiny ? grid_tiny * kTinyWaves * kTinySlab : 0) +
                        (n_small ? grid_small * kSmallSlab : 0) + 2 * int64_t(n_cu_) * kSmallSlab;  // (+ k_srb_row)
  int64_t cap = std::min<int64_t>(bound + slack, est_nnz + est_nnz / 4 + slack);
  const int64_t budget = int64_t((free_b + col_.cap + cnt_.cap) / 10 * 8 / 8);
  cap = std::max<int64_t>(1, std::min(cap, budget));
  dense_mode_ = false;
  last_rows_ = M;
  COOC_TRY(bump_.reserve(sizeof(uint64_t) * 2));
  SpArgs proto{};
  proto.queue = sp_queue_.as<SpWork>();
  proto.tot = tot;
  proto.qctr = qctr;
  proto.vals = vals;
  proto.tb = sp_tb_.as<int32_t>();
  proto.tarena = sp_arena_.as<uint4>();
  proto.tarena0 = sp_arena0_.as<uint4>();
  proto.epre = epre;
  proto.gmass = gmass;
  proto.split_slot = split_slot_.as<int32_t>();
  proto.bump = bump_.as<unsigned long long>();
  proto.slab = slab;
  proto.row_base = row_base_.as<int64_t>();
  proto.row_nnz = row_nnz_.as<int32_t>();
  proto.M = Mc;  // (k_sp_main's column range)
  proto.T = T;
  proto.n_contrib = n_c;
  proto.n_users = U;
  proto.n_groups = n_groups1;
  proto.n_groups0 = n_groups0;
  proto.scratch = scr_cap ? sp_scr_.as<uint4>() : nullptr;
  proto.scr_cap = (scr_cap && n_gather) ? scr_cap : 0;
  proto.rowsum = rowsum_.as<int64_t>();
  proto.spre = spre;
  COOC_TRY(sp_defer_.reserve(sizeof(int32_t) * size_t(M)));
  proto.deferred = sp_defer_.as<int32_t>();
  proto.sort_all = sort_rows_ ? 1 : 0;
  proto.any_order = (any_order_ && !win) ? 1 : 0;
  proto.hot_col = hot_col;
  proto.pos_of = pos_of;
  int64_t last_err = 0;
  for (int attempt = 0; attempt < 2; attempt++) {
    COOC_TRY(col_.reserve(sizeof(int32_t) * size_t(cap + 1)));
    COOC_TRY(cnt_.reserve(sizeof(uint32_t) * size_t(cap + 1)));
    if (n_split > 0)
      COOC_HIP_TRY(hipMemsetAsync(staging_.p, 0, sizeof(uint32_t) * size_t(n_split) * size_t(sstride), s));
    k_sp_reset_run<<<1, 1, 0, s>>>(tot, qctr, bump_.as<unsigned long long>());
    SpArgs A = proto;
    A.staging = staging_.as<uint32_t>();
    A.sstride = sstride;
    A.col_out = col_.as<int32_t>();
    A.cnt_out = cnt_.as<uint32_t>();
    A.cap = cap;
#ifdef COOC_SP_TRACE
    static unsigned long long *prog = nullptr;
    if (!prog) hipHostMalloc(reinterpret_cast<void **>(&prog), 8 * 64 * 1024, hipHostMallocDefault);
    memset(prog, 0xff, 8 * 64 * 1024);
    prog[2047] = 0;
    prog[1024] = 0;
    prog[1536] = 0;
    A.prog = prog;
    fprintf(stderr, "[sp] n_work %lld cap %lld slab %lld est %lld bound %lld\n", (long long)n_work, (long long)cap, (long long)slab, (long long)est_nnz, (long long)bound);
#endif
#ifdef COOC_SP_STATS
    static unsigned long long *d_stats = nullptr;
    if (!d_stats) (void)hipMalloc(reinterpret_cast<void **>(&d_stats), 128 * 8);
    (void)hipMemsetAsync(d_stats, 0, 128 * 8, s);
    A.stats = d_stats;
    A.exp = getenv("COOC_SP_EXP") ? atoi(getenv("COOC_SP_EXP")) : 0;
#endif
    if (timer && timer->enabled) COOC_HIP_TRY(hipEventRecord(timer->acc_begin, s));
    // the mid and small/tiny launches fork onto streams of their own (after everything before on s) and join
    // s again before the span ends; the big launch is issued first, so its workgroups take the CUs first
    const bool fork = fork_mode_ != 0 && (n_mid > 0 || n_small > 0 || n_tiny > 0);
    hipStream_t s_mid = s, s_small = s;
    if (fork) {
      if (!ev_fork_) {
        COOC_HIP_TRY(hipEventCreateWithFlags(&ev_fork_, hipEventDisableTiming));
        for (int i = 0; i < 2; i++) {
          COOC_HIP_TRY(hipStreamCreateWithFlags(&aux_[i], hipStreamNonBlocking));
          COOC_HIP_TRY(hipEventCreateWithFlags(&ev_join_[i], hipEventDisableTiming));
        }
      }
      COOC_HIP_TRY(hipEventRecord(ev_fork_, s));
      s_mid = fork_mode_ == 2 ? s : aux_[0];
      s_small = aux_[1];
    }
    A.q_begin = 0;
    A.q_end = n_big;
    if (n_big > 0) {
      k_sp_main<SpBig><<<unsigned(grid), SpBig::kThreads, SpBig::kLds, s>>>(A);
      COOC_HIP_TRY(hipGetLastError());
#ifdef COOC_SP_TRACE
      for (int it = 0; it < 100 && hipStreamQuery(s) == hipErrorNotReady; it++) usleep(50000);
      if (hipStreamQuery(s) == hipErrorNotReady) {
        for (int g = 0; g < grid; g++)
        {
          fprintf(stderr, "[sp] wg %d: work %lld phase %lld total %lld nb %lld waves", g, (long long)prog[g * 64], (long long)prog[g * 64 + 1], (long long)prog[g * 64 + 2], (long long)prog[g * 64 + 3]);
          for (int w = 0; w < 16; w++) fprintf(stderr, " %lld", (long long)prog[g * 64 + 16 + w]);
          fprintf(stderr, "\n");
        }
        for (int tt = 0; tt < 2; tt++) {
          const unsigned long long *q = prog + 1024 + tt * 512;
          fprintf(stderr, "[sp] thread %d trace (%llu):", tt * 64, q[0]);
          for (unsigned long long i = 0; i < q[0] && i < 255; i++) fprintf(stderr, " %llu", q[1 + i]);
          fprintf(stderr, "\n");
        }
        fflush(stderr);
        _exit(3);
      }
      hipStreamSynchronize(s);
      fprintf(stderr, "[sp] bounds flags %llx\n", prog[2047]);
#endif
    }
    if (n_mid > 0) {  // the mid rows (after the big launch: it holds the heaviest rows)
      SpArgs B = A;
      B.qctr = qctr + 1;
      B.q_begin = n_big;
      B.q_end = n_big + n_mid;
      B.scratch = scr_cap_mid ? sp_scr_mid_.as<uint4>() : nullptr;
      B.scr_cap = (scr_cap_mid && n_gather) ? scr_cap_mid : 0;
#ifdef COOC_SP_STATS
      B.stats = A.stats + 64;
#endif
      if (fork && fork_mode_ == 2) COOC_HIP_TRY(hipEventRecord(ev_fork_, s));  // (after the big launch)
      if (fork && s_mid != s) COOC_HIP_TRY(hipStreamWaitEvent(s_mid, ev_fork_, 0));
      k_sp_main<SpMid><<<unsigned(grid_mid), SpMid::kThreads, SpMid::kLds, s_mid>>>(B);
      COOC_HIP_TRY(hipGetLastError());
    }
    if (fork && (n_small > 0 || n_tiny > 0)) COOC_HIP_TRY(hipStreamWaitEvent(s_small, ev_fork_, 0));
    if (n_small > 0) {
      k_sp_small<<<unsigned(grid_small), kSmallThreads, 0, s_small>>>(A);
      COOC_HIP_TRY(hipGetLastError());
    }
    if (n_tiny > 0) {
      k_sp_tiny<<<unsigned(grid_tiny), kTinyThreads, 0, s_small>>>(A);
      COOC_HIP_TRY(hipGetLastError());
    }
  SPT("main");
    if (n_split > 0) {
      k_sp_split_finalize<<<unsigned(n_split), kFinThreads, 0, s>>>(
          split_row_.as<int32_t>(), staging_.as<uint32_t>(), sstride, Mc, row_ptr, rowsum_.as<int64_t>(), col_.as<int32_t>(),
          cnt_.as<uint32_t>(), bump_.as<unsigned long long>(), cap, row_base_.as<int64_t>(), row_nnz_.as<int32_t>(),
          tot, spre, hot_col, pos_of);
      COOC_HIP_TRY(hipGetLastError());
    }
    if (fork) {  // s waits for the forked launches
      COOC_HIP_TRY(hipEventRecord(ev_join_[0], s_mid));
      COOC_HIP_TRY(hipEventRecord(ev_join_[1], s_small));
      COOC_HIP_TRY(hipStreamWaitEvent(s, ev_join_[0], 0));
      COOC_HIP_TRY(hipStreamWaitEvent(s, ev_join_[1], 0));
    }
    // (the timed span: every counting kernel of the run -- k_sp_main, k_sp_small, k_sp_tiny, the split rows'
    // finalize -- so that moving rows between them cannot flatter the kernel time)
    if (timer && timer->enabled) COOC_HIP_TRY(hipEventRecord(timer->acc_end, s));
  SPT("finalize");
    COOC_HIP_TRY(hipMemcpyAsync(h_tot_, tot, sizeof(PlanTotals), hipMemcpyDeviceToHost, s));
    COOC_HIP_TRY(hipStreamSynchronize(s));
    int64_t err = h_tot_->err;
    const int64_t n_def = h_tot_->n_deferred;
    // (COOC_FLAG_SORT_ROWS: every whole row is sorted -- the tiny and small rows by k_sp_tiny / k_sp_small, the
    // others by the sort path)
    last_deferred_ = n_def + (sort_rows_ ? h_tot_->n_tiny + h_tot_->n_small : 0);
    last_deferred_pairs_ = sort_rows_ ? h_tot_->ts_pairs : 0;
    if (n_def > 0 && !(err & 4)) {  // rows whose hash table overflowed (all whole rows: COOC_FLAG_SORT_ROWS)
      COOC_TRY(run_deferred(n_def, T, row_ptr, epre, vals, spre, cap, s));
      COOC_HIP_TRY(hipMemcpyAsync(&err, &tot->err, sizeof(int64_t), hipMemcpyDeviceToHost, s));
      COOC_HIP_TRY(hipStreamSynchronize(s));
    }
  SPT("deferred");
    k_sp_nnz_total<<<std::min<unsigned>(nblocks(M, 256), 64), 256, 0, s>>>(row_nnz_.as<int32_t>(), M, tot);
    COOC_HIP_TRY(hipGetLastError());
#ifdef COOC_SP_STATS
    {
      unsigned long long hh[128];
      (void)hipMemcpy(hh, A.stats, sizeof(hh), hipMemcpyDeviceToHost);
      for (int shape = 0; shape < 2; shape++) {
      const unsigned long long *h = hh + 64 * shape;
      const double g = double(shape ? grid_mid : grid);
      if (shape && !n_mid) break;
      fprintf(stderr, "[sp stats] %s shape (%lld WGs):\n", shape ? "mid" : "big", (long long)(shape ? grid_mid : grid));
      fprintf(stderr, "[sp stats] per WG (us): total %.0f walk dense %.0f walk hash %.0f split %.0f compact dense %.0f "
              "compact hash %.0f | chunks dense %llu hash %llu overflows %llu deferred rows %llu | pairs dense %.3g hash %.3g | "
              "rows %llu split items %llu | mean H %.0f | tail sizes %.0f\n",
              h[13] / 100.0 / g, h[0] / 100.0 / g, h[1] / 100.0 / g, h[4] / 100.0 / g, h[2] / 100.0 / g, h[3] / 100.0 / g,
              h[5], h[6], h[7], h[8], double(h[9]), double(h[10]), h[11], h[12], h[6] ? double(h[14]) / h[6] : 0.0,
              h[15] / 100.0 / g);
      fprintf(stderr, "[sp stats] hash detail per WG (us): walk scan %.0f walk loop %.0f | groups %.3g batches %llu | "
              "compact rank %.0f reserve %.0f write %.0f | entries %.3g\n", h[16] / 100.0 / g, h[17] / 100.0 / g,
              double(h[18]), h[19], h[20] / 100.0 / g, h[21] / 100.0 / g, h[22] / 100.0 / g, double(h[23]));
      fprintf(stderr, "[sp stats] split flush (staging atomics) per WG (us): %.0f\n", h[26] / 100.0 / g);
      fprintf(stderr, "[sp stats] hash compaction cumulative (us/WG): table+L1 %.0f, +masks %.0f | dense compaction "
              "cumulative (us/WG): count %.0f, +reserve %.0f, +writes %.0f, +barrier %.0f | hash walk: first group "
              "applied after %.2f us (thread 0, %llu walks)\n", h[46] / 100.0 / g, h[47] / 100.0 / g, h[48] / 100.0 / g,
              h[49] / 100.0 / g, h[50] / 100.0 / g, h[51] / 100.0 / g, h[55] ? h[54] / 100.0 / double(h[55]) : 0.0, h[55]);
      fprintf(stderr, "[sp stats] thread-0 sample: ids inserted %llu, probe rounds %llu (%.2f per group call)\n", h[24], h[25],
              h[24] ? double(h[25]) / double(h[24]) * 4.0 : 0.0);
      for (int c = 0; c < 3; c++) {
        const unsigned long long *q = h + 28 + 6 * c;
        fprintf(stderr, "[sp stats] hash class %s: chunks %llu, walk %.0f us/WG (%.2f us/chunk), compact %.0f us/WG "
                "(%.2f us/chunk), groups/chunk %.0f, row entries so far/chunk %.0f, contributions/chunk %.0f\n",
                c == 0 ? "light-row" : c == 1 ? "gathered" : "list-walk", q[0], q[1] / 100.0 / g,
                q[0] ? q[1] / 100.0 / double(q[0]) : 0.0, q[2] / 100.0 / g, q[0] ? q[2] / 100.0 / double(q[0]) : 0.0,
                q[0] ? double(q[3]) / q[0] : 0.0, q[0] ? double(q[4]) / q[0] : 0.0, q[0] ? double(q[5]) / q[0] : 0.0);
      }
      }
      fprintf(stderr, "[sp stats] attempt %d: cap %lld slab %lld grid %lld err %lld scr_cap %lld n_gather %lld\n", attempt,
              (long long)cap, (long long)slab, (long long)grid, (long long)err, (long long)A.scr_cap, (long long)n_gather);
    }
#endif
#ifdef COOC_SP_STATS
    if (A.exp && (err & 2)) {  // (timing experiments drop ids on purpose: the row-sum checks fail)
      err &= ~int64_t(2);
      COOC_HIP_TRY(hipMemcpy(&tot->err, &err, sizeof(int64_t), hipMemcpyHostToDevice));
    }
#endif
    last_err = err;
    if (!(err & 4) || cap >= bound + slack) break;
    // the expected key count was too low: rerun into a region of the exact bound
    size_t f2 = 0, t2 = 0;
    COOC_HIP_TRY(hipMemGetInfo(&f2, &t2));
    const int64_t budget2 = int64_t((f2 + col_.cap + cnt_.cap) / 10 * 8 / 8);
    if (budget2 <= cap) break;
    cap = std::min<int64_t>(bound + slack, budget2);
  }
  if (last_err & 4)  // rows were cut short: never hand out a partial result
    return Status{4, "the output region (" + std::to_string(cap) + " entries) was exhausted"};
  out->row_base = row_base_.as<int64_t>();
  out->row_nnz = row_nnz_.as<int32_t>();
  out->col = col_.as<int32_t>();
  out->cnt = cnt_.as<uint32_t>();
  out->dense = nullptr;
  out->rowsum = rowsum_.as<int64_t>();
  out->rank_of = pos_of;
  out->unordered = proto.any_order != 0;
  out->work = work_total;
  out->observed = work_total - self_total;  // ordered pairs of the counted rows
  out->nnz = -1;  // known after the stream drains: read_totals().nnz_total
  return Status::Ok();
}

// The deferred rows (k_sp_main: hash table overflow; COOC_FLAG_SORT_ROWS: every whole row) through the sort +
// segmented-reduce path, in batches of at most kSrBatchPairs pairs (a whole row has <= kSplitWork).
Status Counter::run_deferred(int64_t n_def, int32_t T, const int64_t *row_ptr, const int64_t *epre,
                             const uint32_t *vals, const int64_t *spre, int64_t cap, hipStream_t s) {
  const int32_t *rows = sp_defer_.as<int32_t>();
  // the rows' pair work (sp_roww_), to the host in deferral order
  COOC_TRY(sr_aux_.reserve(sizeof(int64_t) * size_t(3 * n_def + 8)));
  int64_t *d_w = sr_aux_.as<int64_t>();
  k_sr_pair_work<<<nblocks(n_def, 256), 256, 0, s>>>(rows, n_def, sp_roww_.as<int64_t>(), d_w);
  COOC_HIP_TRY(hipGetLastError());
  std::vector<int64_t> w(size_t(n_def), 0);
  COOC_HIP_TRY(hipMemcpyAsync(w.data(), d_w, sizeof(int64_t) * size_t(n_def), hipMemcpyDeviceToHost, s));
  COOC_HIP_TRY(hipStreamSynchronize(s));
  size_t f0 = 0, t0 = 0;
  COOC_HIP_TRY(hipMemGetInfo(&f0, &t0));
  // 28 B per pair (two key buffers, run keys, run counts); a batch holds any whole row
  int64_t budget = std::min<int64_t>(int64_t(1) << 27, int64_t(f0 / 4 / 28));
  budget = std::max<int64_t>(budget, kSplitWork);
  int64_t max_batch = 0;
  for (int64_t j0 = 0, acc = 0, j = 0; j <= n_def; j++) {  // the largest batch, for the buffers
    if (j == n_def || (acc + w[size_t(j)] > budget && j > j0)) {
      max_batch = std::max(max_batch, acc);
      if (j == n_def) break;
      j0 = j;
      acc = 0;
    }
    acc += w[size_t(j)];
  }
  const int64_t nk = std::max<int64_t>(max_batch, 1);
  if (!srb_hipcub_) {
    // the hand-written path (k_srb_row): persistent workgroups (two per CU) take the rows in deferral order;
    // each has a scratch range for the largest row's pairs as u32 ids + u32 run counts
    int64_t max_w = 1;
    for (int64_t j = 0; j < n_def; j++) {
      max_w = std::max(max_w, w[size_t(j)]);
      last_deferred_pairs_ += w[size_t(j)];
    }
    const int64_t stride = (max_w + 63) & ~int64_t(63);
    int64_t grid = std::min<int64_t>(n_def, 2 * int64_t(n_cu_));
    grid = std::max<int64_t>(1, std::min<int64_t>(grid, int64_t(f0 / 2) / (8 * stride)));
    COOC_TRY(sr_keys_.reserve(sizeof(uint32_t) * size_t(2 * grid * stride)));
    uint32_t *ids = sr_keys_.as<uint32_t>(), *cn = ids + grid * stride;
    unsigned long long *srb_st = nullptr;
#ifdef COOC_SP_STATS
    static unsigned long long *d_srb = nullptr;
    if (!d_srb) COOC_HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_srb), 16 * 8));
    COOC_HIP_TRY(hipMemsetAsync(d_srb, 0, 16 * 8, s));
    srb_st = d_srb;
#endif
    PlanTotals *tot = tot_.as<PlanTotals>();
    COOC_HIP_TRY(hipMemsetAsync(&tot->srb_ctr, 0, sizeof(int64_t), s));
    k_srb_row<<<unsigned(grid), kSrbThreads, 0, s>>>(
        rows, n_def, stride, row_ptr, vals, sp_tb_.as<int32_t>(), sp_arena0_.as<uint16_t>(), sp_arena_.as<uint32_t>(), T,
        last_mc_, ids, cn, spre, rowsum_.as<int64_t>(), last_hot_col_, last_pos_of_, col_.as<int32_t>(),
        cnt_.as<uint32_t>(), bump_.as<unsigned long long>(), cap, row_base_.as<int64_t>(), row_nnz_.as<int32_t>(), tot,
        srb_st);
    COOC_HIP_TRY(hipGetLastError());
#ifdef COOC_SP_STATS
    {
      unsigned long long h[16];
      COOC_HIP_TRY(hipMemcpy(h, srb_st, sizeof(h), hipMemcpyDeviceToHost));
      const double r = h[5] ? double(h[5]) : 1.0;
      fprintf(stderr, "[srb stats] rows %llu contributions %llu pairs %llu | per row (us): hist %.1f partition %.1f "
              "sort groups %.1f (%llu) counting %.1f (%llu) output %.1f total %.1f\n", h[5], h[6], h[7], h[0] / 100.0 / r,
              h[1] / 100.0 / r, h[2] / 100.0 / r, h[8], h[3] / 100.0 / r, h[9], h[4] / 100.0 / r, h[10] / 100.0 / r);
    }
#endif
    return Status::Ok();
  }
  COOC_TRY(sr_keys_.reserve(sizeof(uint64_t) * size_t(2 * nk)));
  COOC_TRY(sr_ukeys_.reserve(sizeof(uint64_t) * size_t(nk)));
  COOC_TRY(sr_ucnt_.reserve(sizeof(uint32_t) * size_t(nk)));
  uint64_t *keys = sr_keys_.as<uint64_t>(), *keys2 = keys + nk, *ukeys = sr_ukeys_.as<uint64_t>();
  uint32_t *ucnt = sr_ucnt_.as<uint32_t>();
  int64_t *n_runs = d_w + n_def;  // [1]; then kbase [nb + 1], rstart [nb + 1] after it
  int64_t *kbase = n_runs + 2;
  size_t tmp = 0, q = 0;
  COOC_HIP_TRY(hipcub::DeviceRadixSort::SortKeys(nullptr, q, keys, keys2, int(nk), 0, 64, s));
  tmp = std::max(tmp, q);
  COOC_HIP_TRY(hipcub::DeviceRunLengthEncode::Encode(nullptr, q, keys2, ukeys, ucnt, n_runs, int(nk), s));
  tmp = std::max(tmp, q);
  COOC_TRY(sort_tmp_.reserve(tmp));
  std::vector<int64_t> kb;
  int64_t j0 = 0;
  while (j0 < n_def) {
    int64_t j1 = j0, acc = 0;
    kb.assign(1, 0);
    while (j1 < n_def && (j1 == j0 || acc + w[size_t(j1)] <= budget)) {
      acc += w[size_t(j1)];
      kb.push_back(acc);
      j1++;
    }
    const int32_t nb = int32_t(j1 - j0);
    last_deferred_pairs_ += acc;
    if (acc > 0) {
      int64_t *rstart = kbase + (nb + 1);
      COOC_HIP_TRY(hipMemcpyAsync(kbase, kb.data(), sizeof(int64_t) * size_t(nb + 1), hipMemcpyHostToDevice, s));
      k_sr_expand<<<unsigned(nb), kSrThreads, 0, s>>>(rows + j0, kbase, row_ptr, epre, vals, sp_tb_.as<int32_t>(),
                                                      sp_arena0_.as<uint16_t>(), sp_arena_.as<uint32_t>(), T, keys);
      COOC_HIP_TRY(hipGetLastError());
      size_t b = sort_tmp_.cap;
      COOC_HIP_TRY(hipcub::DeviceRadixSort::SortKeys(sort_tmp_.p, b, keys, keys2, int(acc), 0, 32 + bits_for(nb + 1), s));
      b = sort_tmp_.cap;
      COOC_HIP_TRY(hipcub::DeviceRunLengthEncode::Encode(sort_tmp_.p, b, keys2, ukeys, ucnt, n_runs, int(acc), s));
      k_sr_bounds<<<nblocks(nb + 1, 256), 256, 0, s>>>(ukeys, n_runs, nb, rstart);
      k_sr_emit<<<unsigned(nb), kSrThreads, 0, s>>>(rows + j0, rstart, ukeys, ucnt, row_ptr, spre, rowsum_.as<int64_t>(),
                                                    col_.as<int32_t>(), cnt_.as<uint32_t>(), bump_.as<unsigned long long>(),
                                                    cap, row_base_.as<int64_t>(), row_nnz_.as<int32_t>(),
                                                    tot_.as<PlanTotals>(), last_hot_col_, last_pos_of_);
      COOC_HIP_TRY(hipGetLastError());
      // kb (host) is reused by the next batch's upload: the copy must have been consumed
      COOC_HIP_TRY(hipStreamSynchronize(s));
    }
    j0 = j1;
  }
  return Status::Ok();
}

}  // namespace cooc
