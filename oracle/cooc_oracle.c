/*
 * cooc_oracle.c — CPU restatement of the reference's non-sampled co-occurrence path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP product path.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product
 * library (flink-cooccurrence_amd/csrc) never links or calls it.
 *
 * Parity status: the LLR and the priority queue are pinned by the reference's own known-answer
 * tests (LogLikelihoodTest.java:14-16, IntDoublePriorityQueueTest.java:12-98; see
 * tests/test_oracle_kat.py).  The reference ships NO fixture for pair counts, row sums or
 * windows and cannot run here (Java/Flink/fastutil absent), so count
 * parity is "parity unpinned" by the reference: it is pinned only by hand-derived micro-logs
 * (tests/golden/micro_logs.json) and by agreement with an independent closed form
 * (C = A^T A - diag(colsum A), oracle/oracle.py).
 *
 * Everything below restates /root/reference/src/main/java/com/github/uce/flinkcooccurrences/
 *   NonSampledUserInteractionCounterOneInputStreamOperator.java (abbrev. NonSampled)
 *   ItemCooccurrences.java, ItemRowAggregator.java, RowSumAggregator.java,
 *   ItemRowRescorerTwoInputStreamOperator.java (abbrev. Rescorer), LogLikelihood.java,
 *   IntDoublePriorityQueue.java
 * record by record (O(P) work), not in closed form.
 *
 * Third-party semantics restated (not in /root/reference, Maven deps of pom.xml:64-74):
 *   fastutil 8.1.0 Int2ShortOpenHashMap.addTo: value += (short) increment with int16 wrap,
 *     key kept even when the value returns to 0, get() of a missing key = 0.
 *   fastutil Int2IntOpenHashMap.addTo/get: int32 wrap, default 0.
 *   Flink 1.3.2 TumblingEventTimeWindows (offset 0): start = ts - (ts + size) % size (Java %),
 *     maxTimestamp = start + size - 1; an event-time timer fires when watermark >= its time.
 *   java.util.Random: 48-bit LCG, multiplier 0x5DEECE66D, addend 0xB.
 *
 * Iteration order: fastutil's hash-slot order is not reproducible without fastutil, so rows
 * are iterated in ascending column order here and in the HIP path (documented tie contract,
 * SURVEY.md §8(a) item 4).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------------------------------------ */
/* int32 -> slot hash (open addressing, linear probing).                                       */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  int32_t *keys;
  int32_t *slot; /* value: an index into caller-owned arrays, -1 = empty */
  int64_t cap;   /* power of two */
  int64_t n;
} i32map;

static uint32_t mix32(uint32_t x) { /* murmur3 finaliser; order only matters for speed */
  x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16;
  return x;
}

static void i32map_init(i32map *m, int64_t cap) {
  int64_t c = 16;
  while (c < cap * 2) c <<= 1;
  m->keys = (int32_t *)malloc(sizeof(int32_t) * c);
  m->slot = (int32_t *)malloc(sizeof(int32_t) * c);
  for (int64_t i = 0; i < c; i++) m->slot[i] = -1;
  m->cap = c;
  m->n = 0;
}

static void i32map_free(i32map *m) { free(m->keys); free(m->slot); m->keys = NULL; m->slot = NULL; }

static int32_t i32map_get(const i32map *m, int32_t key) {
  uint64_t mask = (uint64_t)m->cap - 1, i = mix32((uint32_t)key) & mask;
  while (m->slot[i] >= 0) {
    if (m->keys[i] == key) return m->slot[i];
    i = (i + 1) & mask;
  }
  return -1;
}

static void i32map_put_new(i32map *m, int32_t key, int32_t value);

static void i32map_grow(i32map *m) {
  i32map g;
  i32map_init(&g, m->cap);
  for (int64_t i = 0; i < m->cap; i++)
    if (m->slot[i] >= 0) i32map_put_new(&g, m->keys[i], m->slot[i]);
  i32map_free(m);
  *m = g;
}

static void i32map_put_new(i32map *m, int32_t key, int32_t value) {
  if ((m->n + 1) * 2 > m->cap) i32map_grow(m);
  uint64_t mask = (uint64_t)m->cap - 1, i = mix32((uint32_t)key) & mask;
  while (m->slot[i] >= 0) i = (i + 1) & mask;
  m->keys[i] = key;
  m->slot[i] = value;
  m->n++;
}

/* ------------------------------------------------------------------------------------------ */
/* Row map = Int2ShortOpenHashMap restatement with an exact int64 shadow per key.              */
/* ItemRowAggregator.java:21-31 (per-window accumulator), Rescorer:172-177 (global row).       */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  i32map idx;
  int32_t *col;
  int16_t *v16;   /* the reference's value: short, wraps (fastutil addTo) */
  int64_t *exact; /* the exact count the GPU path also exposes */
  int32_t n, cap;
} rowmap;

static void rowmap_init(rowmap *r) {
  i32map_init(&r->idx, 8); /* new Int2ShortOpenHashMap(8), ItemRowAggregator.java:22 */
  r->cap = 8;
  r->n = 0;
  r->col = (int32_t *)malloc(sizeof(int32_t) * r->cap);
  r->v16 = (int16_t *)malloc(sizeof(int16_t) * r->cap);
  r->exact = (int64_t *)malloc(sizeof(int64_t) * r->cap);
}

static void rowmap_free(rowmap *r) {
  i32map_free(&r->idx);
  free(r->col); free(r->v16); free(r->exact);
}

/* fastutil addTo: (short)(old + incr); key retained even when it becomes 0. */
static void rowmap_add_to(rowmap *r, int32_t col, int16_t incr16, int64_t incr_exact) {
  int32_t s = i32map_get(&r->idx, col);
  if (s < 0) {
    if (r->n == r->cap) {
      r->cap *= 2;
      r->col = (int32_t *)realloc(r->col, sizeof(int32_t) * r->cap);
      r->v16 = (int16_t *)realloc(r->v16, sizeof(int16_t) * r->cap);
      r->exact = (int64_t *)realloc(r->exact, sizeof(int64_t) * r->cap);
    }
    s = r->n++;
    r->col[s] = col;
    r->v16[s] = 0;
    r->exact[s] = 0;
    i32map_put_new(&r->idx, col, s);
  }
  r->v16[s] = (int16_t)(uint16_t)((uint16_t)r->v16[s] + (uint16_t)incr16);
  r->exact[s] += incr_exact;
}

static int cmp64(const void *p, const void *q) {
  int64_t x = *(const int64_t *)p, y = *(const int64_t *)q;
  return (x > y) - (x < y);
}

/* Entry order of a row in ascending column (the documented iteration order). */
static int32_t *rowmap_sorted_slots(const rowmap *r) {
  /* sort (col, slot) pairs packed into int64 */
  int64_t *tmp = (int64_t *)malloc(sizeof(int64_t) * (r->n ? r->n : 1));
  for (int32_t i = 0; i < r->n; i++) tmp[i] = ((int64_t)r->col[i] << 32) | (uint32_t)i;
  /* columns are non-negative item ids, so signed order == column order */
  qsort(tmp, (size_t)r->n, sizeof(int64_t), cmp64);
  int32_t *slots = (int32_t *)malloc(sizeof(int32_t) * (r->n ? r->n : 1));
  for (int32_t i = 0; i < r->n; i++) slots[i] = (int32_t)(uint32_t)(tmp[i] & 0xffffffff);
  free(tmp);
  return slots;
}

/* ------------------------------------------------------------------------------------------ */
/* LogLikelihood.java:41-61 (9-log form).  Compiled with -ffp-contract=off: Java never fuses.  */
/* ------------------------------------------------------------------------------------------ */
/* Math.log as Java's StrictMath.log pins it: fdlibm 5.3's __ieee754_log (e_log.c; the JDK's StrictMath.log is
 * that function, and Java's Math.log may differ from it by at most an ulp).  Third-party arithmetic, not in
 * /root/reference: restated from fdlibm's published method -- x = 2^k (1 + f) with sqrt(2)/2 < 1 + f < sqrt(2),
 * s = f / (2 + f), log(1 + f) = f - s (f - R(s^2)) with fdlibm's degree-14 Remez polynomial R (Lg1..Lg7), and
 * k ln2 split in ln2_hi + ln2_lo -- in its operation order.  The device's rescoring kernel computes the same
 * function (cooc_stream.hip, java_log), so every LLR score is reproducible bit for bit. */
static double strict_log(double x) {
  static const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                      two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
                      Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                      Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01,
                      Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
  union { double d; uint64_t u; } v = {x};
  int32_t hx = (int32_t)(v.u >> 32);
  const uint32_t lx = (uint32_t)v.u;
  int32_t k = 0;
  if (hx < 0x00100000) {                           /* x < 2^-1022 */
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -INFINITY;  /* log(+-0) */
    if (hx < 0) return NAN;                         /* log(negative) */
    k -= 54;                                        /* subnormal: scale up */
    v.d *= two54;
    hx = (int32_t)(v.u >> 32);
  }
  if (hx >= 0x7ff00000) return v.d + v.d;          /* inf or NaN */
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  const int32_t i0 = (hx + 0x95f64) & 0x100000;
  v.u = ((uint64_t)(uint32_t)(hx | (i0 ^ 0x3ff00000)) << 32) | (v.u & 0xffffffffu); /* x or x/2 into [sqrt2/2, sqrt2) */
  k += i0 >> 20;
  const double f = v.d - 1.0;
  if ((0x000fffff & (2 + hx)) < 3) {               /* |f| < 2^-20 */
    if (f == 0.0) {
      if (k == 0) return 0.0;
      const double dk = (double)k;
      return dk * ln2_hi + dk * ln2_lo;
    }
    const double R = f * f * (0.5 - 0.33333333333333333 * f);
    if (k == 0) return f - R;
    const double dk = (double)k;
    return dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  const double s = f / (2.0 + f);
  const double dk = (double)k;
  const double z = s * s;
  int32_t i = hx - 0x6147a;
  const double w = z * z;
  const int32_t j = 0x6b851 - hx;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  i |= j;
  const double R = t2 + t1;
  if (i > 0) {
    const double hfsq = 0.5 * f * f;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  if (k == 0) return f - s * (f - R);
  return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

EXPORT double oc_strict_log(double x) { return strict_log(x); }

static double xlogx(int64_t x) { /* LogLikelihood.java:59-61 */
  return x == 0 ? 0.0 : (double)x * strict_log((double)x);
}

EXPORT double oc_llr(int64_t k11, int64_t k12, int64_t k21, int64_t k22) {
  const int64_t k11k12 = k11 + k12; /* :43 */
  const int64_t k21k22 = k21 + k22; /* :44 */
  const double all = xlogx(k11k12 + k21k22);                                         /* :46 */
  const double row = all - xlogx(k11k12) - xlogx(k21k22);                            /* :47 */
  const double column = all - xlogx(k11 + k21) - xlogx(k12 + k22);                   /* :48 */
  const double matrix = all - xlogx(k11) - xlogx(k12) - xlogx(k21) - xlogx(k22);     /* :49 */
  if (row + column < matrix) return 0.0;                                             /* :51-53 */
  return 2.0 * (row + column - matrix);                                              /* :55 */
}

/* Rescorer.scoreItem, ItemRowRescorerTwoInputStreamOperator.java:230-241 */
EXPORT double oc_score_item(int16_t k11, int64_t item_row_sum, int64_t other_row_sum, int64_t observed) {
  const int64_t k12 = item_row_sum - k11;
  const int64_t k21 = other_row_sum - k11;
  const int64_t k22 = observed + k11 - k12 - k21; /* :238, non-standard on purpose */
  return oc_llr(k11, k12, k21, k22);
}

/* ------------------------------------------------------------------------------------------ */
/* IntDoublePriorityQueue.java:48-205 (Lucene-style 1-based min-heap)                          */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  int32_t *values;
  double *scores;
  int32_t size, max_size;
} oc_pq;

EXPORT oc_pq *oc_pq_create(int32_t max_size) { /* :69-78 */
  if (max_size < 1) return NULL;
  oc_pq *q = (oc_pq *)calloc(1, sizeof(oc_pq));
  q->values = (int32_t *)calloc((size_t)max_size + 1, sizeof(int32_t));
  q->scores = (double *)calloc((size_t)max_size + 1, sizeof(double));
  q->max_size = max_size;
  return q;
}

EXPORT void oc_pq_destroy(oc_pq *q) { if (q) { free(q->values); free(q->scores); free(q); } }
EXPORT int32_t oc_pq_size(const oc_pq *q) { return q->size; }
EXPORT int32_t oc_pq_least_value(const oc_pq *q) { return q->values[1]; } /* :98-100 */
EXPORT double oc_pq_least_score(const oc_pq *q) { return q->scores[1]; }  /* :111-113 */
EXPORT void oc_pq_reset(oc_pq *q) { q->size = 0; }                        /* :120-122 */

static void pq_up_heap(oc_pq *q, int32_t orig) { /* :153-172 */
  int32_t i = orig;
  int32_t value = q->values[i];
  double score = q->scores[i];
  int32_t j = (int32_t)((uint32_t)i >> 1);
  while (j > 0 && score < q->scores[j]) {
    q->values[i] = q->values[j];
    q->scores[i] = q->scores[j];
    i = j;
    j = (int32_t)((uint32_t)j >> 1);
  }
  q->values[i] = value;
  q->scores[i] = score;
}

static void pq_down_heap(oc_pq *q) { /* :174-205 */
  int32_t value = q->values[1];
  double score = q->scores[1];
  int32_t i = 1, j = i << 1, k = j + 1;
  if (k <= q->size && q->scores[k] < q->scores[j]) j = k;
  while (j <= q->size && q->scores[j] < score) {
    q->values[i] = q->values[j];
    q->scores[i] = q->scores[j];
    i = j;
    j = i << 1;
    k = j + 1;
    if (k <= q->size && q->scores[k] < q->scores[j]) j = k;
  }
  q->values[i] = value;
  q->scores[i] = score;
}

/* :132-137; returns -1 where Java would throw ArrayIndexOutOfBoundsException */
EXPORT int oc_pq_add(oc_pq *q, int32_t value, double score) {
  if (q->size >= q->max_size) return -1;
  q->size++;
  q->values[q->size] = value;
  q->scores[q->size] = score;
  pq_up_heap(q, q->size);
  return 0;
}

EXPORT void oc_pq_update(oc_pq *q, int32_t value, double score) { /* :146-150 */
  q->values[1] = value;
  q->scores[1] = score;
  pq_down_heap(q);
}

/* iterator(), :215-242: positions 1..size, least first */
EXPORT void oc_pq_entries(const oc_pq *q, int32_t *values, double *scores) {
  for (int32_t i = 1; i <= q->size; i++) {
    values[i - 1] = q->values[i];
    scores[i - 1] = q->scores[i];
  }
}

/* The caller-side top-k loop of Rescorer:218-222. */
static void pq_offer(oc_pq *q, int32_t topk, int32_t value, double score) {
  if (q->size < topk) oc_pq_add(q, value, score);
  else if (score > q->scores[1]) oc_pq_update(q, value, score);
}

/* ------------------------------------------------------------------------------------------ */
/* java.util.Random (needed to regenerate IntDoublePriorityQueueTest.java:39-43's inputs)       */
/* ------------------------------------------------------------------------------------------ */
static int32_t jr_next(uint64_t *seed, int bits) {
  *seed = (*seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
  return (int32_t)(int64_t)(*seed >> (48 - bits));
}

EXPORT void oc_java_random_doubles(int64_t seed, int32_t n, double *out) {
  uint64_t s = ((uint64_t)seed ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1);
  for (int32_t i = 0; i < n; i++) {
    int64_t hi = (int64_t)(uint32_t)jr_next(&s, 26);
    int64_t lo = (int64_t)(uint32_t)jr_next(&s, 27);
    out[i] = (double)((hi << 27) + lo) * (1.0 / (double)(1ULL << 53));
  }
}

/* Random.nextInt() = next(32) */
EXPORT void oc_java_random_next_int32(int64_t seed, int32_t n, int32_t *out) {
  uint64_t s = ((uint64_t)seed ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1);
  for (int32_t i = 0; i < n; i++) out[i] = jr_next(&s, 32);
}

EXPORT void oc_java_random_ints(int64_t seed, int32_t bound, int32_t n, int32_t *out) {
  uint64_t s = ((uint64_t)seed ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1);
  for (int32_t i = 0; i < n; i++) {
    if ((bound & -bound) == bound) {
      out[i] = (int32_t)(((int64_t)bound * (int64_t)jr_next(&s, 31)) >> 31);
      continue;
    }
    int32_t bits, val;
    do {
      bits = jr_next(&s, 31);
      val = bits % bound;
    } while ((int32_t)((uint32_t)bits - (uint32_t)val + (uint32_t)(bound - 1)) < 0);
    out[i] = val;
  }
}

/* ------------------------------------------------------------------------------------------ */
/* Growable int arrays                                                                          */
/* ------------------------------------------------------------------------------------------ */
typedef struct { int32_t *a; int64_t n, cap; } ivec;
static void ivec_push(ivec *v, int32_t x) {
  if (v->n == v->cap) {
    v->cap = v->cap ? v->cap * 2 : 8;
    v->a = (int32_t *)realloc(v->a, sizeof(int32_t) * v->cap);
  }
  v->a[v->n++] = x;
}

/* ------------------------------------------------------------------------------------------ */
/* Streaming state: NonSampled operator + the two window aggregators + the rescorer           */
/* ------------------------------------------------------------------------------------------ */
typedef struct { /* one pending (window) of NonSampled's keyed ListState windowState, :56,99-100 */
  int64_t max_ts;
  ivec users, items; /* arrival order across keys; per-key order is what matters */
} pending_window;

typedef struct { /* one fired window's observable outputs */
  int64_t ts;                        /* window.maxTimestamp(), NonSampled:115 */
  int32_t n_rows;                    /* delta rows emitted, ItemRowAggregator.java:50-56 */
  int32_t *rows;                     /* ascending item */
  int64_t *row_ptr;                  /* n_rows + 1 */
  int32_t *cols;                     /* ascending within a row */
  int64_t *exact;
  int16_t *v16;
  int32_t n_rowsums;                 /* items with a non-zero exact row-sum delta */
  int32_t *rs_items;
  int64_t *rs_exact;
  int32_t *rs_v32;                   /* RowSumAggregator.java:25-27 int accumulation (wraps) */
  int64_t observed_acc;              /* UserInteractionCounterObservedCooccurrences delta, NonSampled:153 */
  int32_t n_topk;                    /* rescored rows, Rescorer:161-227 */
  int32_t *tk_rows;
  int32_t *tk_sizes;
  int32_t *tk_values;                /* n_topk * topk, heap positions 1..size */
  double *tk_scores;
} fired_window;

typedef struct {
  int64_t window_size;
  int32_t topk;
  int32_t user_cut;  /* kMax, 0 = off: UserInteractionCounter...java:54,168 (deterministic branch only) */
  int64_t watermark; /* timerService.currentWatermark(); starts at Long.MIN_VALUE */
  /* keyed user history, NonSampled:57,129-161 */
  i32map user_idx;
  ivec *hist;
  int32_t n_users, cap_users;
  /* pending windows */
  pending_window *pw;
  int32_t n_pw, cap_pw;
  /* fired outputs */
  fired_window *fw;
  int32_t n_fw, cap_fw;
  /* Rescorer global state, :33-37 */
  i32map grow_idx; /* item -> global row */
  rowmap *grows;
  int32_t n_grows, cap_grows;
  i32map grs_idx;  /* globalItemRowSums (Int2IntOpenHashMap) */
  int32_t *grs_v32;
  int64_t *grs_exact;
  int32_t n_grs, cap_grs;
  int64_t observed_ref;  /* Rescorer:37,154 long += (int) delta */
  /* accumulators */
  int64_t late_elements;     /* NonSampled:79,90 */
  int64_t observed_acc;      /* NonSampled:80,153 */
  int64_t rowsum_acc;        /* RowSumAggregator.java:50,67 */
  int64_t rescored_items;    /* Rescorer:60,169 */
} oc_state;

EXPORT oc_state *oc_create(int64_t window_size, int32_t topk) {
  if (window_size <= 0 || topk < 0) return NULL;
  oc_state *s = (oc_state *)calloc(1, sizeof(oc_state));
  s->window_size = window_size;
  s->topk = topk;
  s->watermark = INT64_MIN;
  i32map_init(&s->user_idx, 1024);
  i32map_init(&s->grow_idx, 1024);
  i32map_init(&s->grs_idx, 1024);
  return s;
}

/* UserInteractionCounter(..., short userCut, ...), :76-81.  Only the `userInteractions < userCut`
 * branch (:168-205) is restated: it is NonSampled's expansion for the first userCut sampled
 * interactions of a user.  The reservoir branch (:206-240, a shared java.util.Random) is replaced by
 * dropping the interaction: the deterministic subset SURVEY.md §8(f).4 names. */
EXPORT int oc_set_user_cut(oc_state *s, int32_t user_cut) {
  if (user_cut < 0 || user_cut > 32767) return 1; /* a Java short */
  s->user_cut = user_cut;
  return 0;
}

static void fired_free(fired_window *f) {
  free(f->rows); free(f->row_ptr); free(f->cols); free(f->exact); free(f->v16);
  free(f->rs_items); free(f->rs_exact); free(f->rs_v32);
  free(f->tk_rows); free(f->tk_sizes); free(f->tk_values); free(f->tk_scores);
}

EXPORT void oc_destroy(oc_state *s) {
  if (!s) return;
  i32map_free(&s->user_idx);
  for (int32_t i = 0; i < s->n_users; i++) free(s->hist[i].a);
  free(s->hist);
  for (int32_t i = 0; i < s->n_pw; i++) { free(s->pw[i].users.a); free(s->pw[i].items.a); }
  free(s->pw);
  for (int32_t i = 0; i < s->n_fw; i++) fired_free(&s->fw[i]);
  free(s->fw);
  i32map_free(&s->grow_idx);
  for (int32_t i = 0; i < s->n_grows; i++) rowmap_free(&s->grows[i]);
  free(s->grows);
  i32map_free(&s->grs_idx);
  free(s->grs_v32); free(s->grs_exact);
  free(s);
}

/* Flink TumblingEventTimeWindows, offset 0 [3P]: start = ts - (ts - 0 + size) % size (Java %). */
EXPORT int64_t oc_window_max_ts(int64_t ts, int64_t size) {
  int64_t start = ts - (ts + size) % size; /* C99 % truncates like Java's */
  return start + size - 1;
}

/* NonSampled.processElement, :84-110.  Returns 1 when the element is late and dropped. */
EXPORT int oc_process_element(oc_state *s, int32_t user, int32_t item, int64_t ts) {
  if (ts <= s->watermark) { /* :89-91 */
    s->late_elements++;
    return 1;
  }
  int64_t max_ts = oc_window_max_ts(ts, s->window_size);
  int32_t w = -1;
  for (int32_t i = 0; i < s->n_pw; i++)
    if (s->pw[i].max_ts == max_ts) { w = i; break; }
  if (w < 0) {
    if (s->n_pw == s->cap_pw) {
      s->cap_pw = s->cap_pw ? s->cap_pw * 2 : 8;
      s->pw = (pending_window *)realloc(s->pw, sizeof(pending_window) * s->cap_pw);
    }
    w = s->n_pw++;
    memset(&s->pw[w], 0, sizeof(pending_window));
    s->pw[w].max_ts = max_ts;
  }
  ivec_push(&s->pw[w].users, user); /* windowState.add(interaction), :99-100 */
  ivec_push(&s->pw[w].items, item);
  return 0;
}

EXPORT int64_t oc_process_elements(oc_state *s, int64_t n, const int32_t *users, const int32_t *items,
                                   const int64_t *ts) {
  int64_t late = 0;
  for (int64_t i = 0; i < n; i++) late += oc_process_element(s, users[i], items[i], ts[i]);
  return late;
}

static ivec *user_history(oc_state *s, int32_t user) { /* userHistoryState.value(), :129-132 */
  int32_t u = i32map_get(&s->user_idx, user);
  if (u < 0) {
    if (s->n_users == s->cap_users) {
      s->cap_users = s->cap_users ? s->cap_users * 2 : 1024;
      s->hist = (ivec *)realloc(s->hist, sizeof(ivec) * s->cap_users);
    }
    u = s->n_users++;
    memset(&s->hist[u], 0, sizeof(ivec));
    i32map_put_new(&s->user_idx, user, u);
  }
  return &s->hist[u];
}

typedef struct { /* per-window aggregation: keyBy(item) + 1-window tumbling windows */
  i32map row_idx;
  rowmap *rows;
  int32_t n_rows, cap_rows;
  i32map rs_idx;
  int32_t *rs_items;
  int32_t *rs_v32;
  int64_t *rs_exact;
  int32_t n_rs, cap_rs;
} window_agg;

static rowmap *agg_row(window_agg *g, int32_t item) { /* createAccumulator, ItemRowAggregator.java:21-23 */
  int32_t r = i32map_get(&g->row_idx, item);
  if (r < 0) {
    if (g->n_rows == g->cap_rows) {
      g->cap_rows = g->cap_rows ? g->cap_rows * 2 : 64;
      g->rows = (rowmap *)realloc(g->rows, sizeof(rowmap) * g->cap_rows);
    }
    r = g->n_rows++;
    rowmap_init(&g->rows[r]);
    i32map_put_new(&g->row_idx, item, r);
  }
  return &g->rows[r];
}

/* RowSumAggregateFunction.add, RowSumAggregator.java:25-27 (int, wraps) */
static void agg_rowsum(window_agg *g, int32_t item, int32_t update) {
  int32_t r = i32map_get(&g->rs_idx, item);
  if (r < 0) {
    if (g->n_rs == g->cap_rs) {
      g->cap_rs = g->cap_rs ? g->cap_rs * 2 : 64;
      g->rs_items = (int32_t *)realloc(g->rs_items, sizeof(int32_t) * g->cap_rs);
      g->rs_v32 = (int32_t *)realloc(g->rs_v32, sizeof(int32_t) * g->cap_rs);
      g->rs_exact = (int64_t *)realloc(g->rs_exact, sizeof(int64_t) * g->cap_rs);
    }
    r = g->n_rs++;
    g->rs_items[r] = item;
    g->rs_v32[r] = 0;
    g->rs_exact[r] = 0;
    i32map_put_new(&g->rs_idx, item, r);
  }
  g->rs_v32[r] = (int32_t)((uint32_t)g->rs_v32[r] + (uint32_t)update);
  g->rs_exact[r] += update;
}

/*
 * NonSampled.onEventTime, :113-165, for one user's interaction: emits the ItemCooccurrences
 * records (as the keyed ItemRowAggregator sees them after the Kryo round trip,
 * ItemCooccurrences.java:116-146: k == -1, so all `size` other items are carried) and the
 * row-sum records.
 */
static void expand_interaction(oc_state *s, window_agg *g, ivec *hist, int32_t item) {
  int64_t size = hist->n; /* :134-135 */
  /* UserInteractionCounter...java:168: userInteractions (= history length here) < userCut */
  if (s->user_cut > 0 && size >= s->user_cut) return;
  if (size > 0) {
    /* :138-139  ITEM (item, history[0..size), +1) -> ItemRowAggregator.add, :26-31 */
    rowmap *r = agg_row(g, item);
    for (int64_t i = 0; i < size; i++) rowmap_add_to(r, hist->a[i], (int16_t)1, 1);
    /* :141-142  ROW_SUM (item, size) */
    agg_rowsum(g, item, (int32_t)size);
    /* :144-151 */
    for (int64_t i = 0; i < size; i++) {
      int32_t other = hist->a[i];
      rowmap_add_to(agg_row(g, other), item, (int16_t)1, 1);
      agg_rowsum(g, other, 1);
    }
    s->observed_acc += 2 * size; /* :153 */
  }
  ivec_push(hist, item); /* :160-161 */
}

static rowmap *global_row(oc_state *s, int32_t item) { /* Rescorer:172 computeIfAbsent */
  int32_t r = i32map_get(&s->grow_idx, item);
  if (r < 0) {
    if (s->n_grows == s->cap_grows) {
      s->cap_grows = s->cap_grows ? s->cap_grows * 2 : 64;
      s->grows = (rowmap *)realloc(s->grows, sizeof(rowmap) * s->cap_grows);
    }
    r = s->n_grows++;
    rowmap_init(&s->grows[r]);
    i32map_put_new(&s->grow_idx, item, r);
  }
  return &s->grows[r];
}

static int32_t global_rowsum_slot(oc_state *s, int32_t item, int create) {
  int32_t r = i32map_get(&s->grs_idx, item);
  if (r < 0 && create) {
    if (s->n_grs == s->cap_grs) {
      s->cap_grs = s->cap_grs ? s->cap_grs * 2 : 64;
      s->grs_v32 = (int32_t *)realloc(s->grs_v32, sizeof(int32_t) * s->cap_grs);
      s->grs_exact = (int64_t *)realloc(s->grs_exact, sizeof(int64_t) * s->cap_grs);
    }
    r = s->n_grs++;
    s->grs_v32[r] = 0;
    s->grs_exact[r] = 0;
    i32map_put_new(&s->grs_idx, item, r);
  }
  return r;
}

static int32_t global_rowsum32(oc_state *s, int32_t item) { /* Int2IntOpenHashMap.get: 0 if absent */
  int32_t r = global_rowsum_slot(s, item, 0);
  return r < 0 ? 0 : s->grs_v32[r];
}

static void fire_window(oc_state *s, pending_window *p) {
  window_agg g;
  memset(&g, 0, sizeof(g));
  i32map_init(&g.row_idx, 64);
  i32map_init(&g.rs_idx, 64);
  int64_t observed_before = s->observed_acc;

  /* NonSampled.onEventTime, :118 iterates windowState in insertion order */
  for (int64_t i = 0; i < p->items.n; i++)
    expand_interaction(s, &g, user_history(s, p->users.a[i]), p->items.a[i]);

  if (s->n_fw == s->cap_fw) {
    s->cap_fw = s->cap_fw ? s->cap_fw * 2 : 8;
    s->fw = (fired_window *)realloc(s->fw, sizeof(fired_window) * s->cap_fw);
  }
  fired_window *f = &s->fw[s->n_fw++];
  memset(f, 0, sizeof(*f));
  f->ts = p->max_ts;
  f->observed_acc = s->observed_acc - observed_before;

  /* ItemCooccurrenceRowWindowFunction.process, ItemRowAggregator.java:50-56: one row per item */
  int32_t *order = (int32_t *)malloc(sizeof(int32_t) * (g.n_rows ? g.n_rows : 1));
  {
    /* rows in ascending item order; the item of row i is recovered from the index map */
    int64_t *tmp = (int64_t *)malloc(sizeof(int64_t) * (g.n_rows ? g.n_rows : 1));
    for (int64_t k = 0; k < g.row_idx.cap; k++)
      if (g.row_idx.slot[k] >= 0) tmp[g.row_idx.slot[k]] = ((int64_t)g.row_idx.keys[k] << 32) | (uint32_t)g.row_idx.slot[k];
    qsort(tmp, (size_t)g.n_rows, sizeof(int64_t), cmp64);
    for (int32_t i = 0; i < g.n_rows; i++) order[i] = (int32_t)(tmp[i] & 0xffffffff);
    f->n_rows = g.n_rows;
    f->rows = (int32_t *)malloc(sizeof(int32_t) * (g.n_rows ? g.n_rows : 1));
    for (int32_t i = 0; i < g.n_rows; i++) f->rows[i] = (int32_t)(tmp[i] >> 32);
    free(tmp);
  }
  int64_t nnz = 0;
  for (int32_t i = 0; i < g.n_rows; i++) nnz += g.rows[i].n;
  f->row_ptr = (int64_t *)malloc(sizeof(int64_t) * (g.n_rows + 1));
  f->cols = (int32_t *)malloc(sizeof(int32_t) * (nnz ? nnz : 1));
  f->exact = (int64_t *)malloc(sizeof(int64_t) * (nnz ? nnz : 1));
  f->v16 = (int16_t *)malloc(sizeof(int16_t) * (nnz ? nnz : 1));
  int64_t pos = 0;
  for (int32_t i = 0; i < g.n_rows; i++) {
    rowmap *r = &g.rows[order[i]];
    int32_t *slots = rowmap_sorted_slots(r);
    f->row_ptr[i] = pos;
    for (int32_t j = 0; j < r->n; j++) {
      f->cols[pos] = r->col[slots[j]];
      f->exact[pos] = r->exact[slots[j]];
      f->v16[pos] = r->v16[slots[j]];
      pos++;
    }
    free(slots);
  }
  f->row_ptr[g.n_rows] = pos;

  /* RowSumProcessWindow.process, RowSumAggregator.java:54-71 */
  {
    int64_t *tmp = (int64_t *)malloc(sizeof(int64_t) * (g.n_rs ? g.n_rs : 1));
    for (int32_t i = 0; i < g.n_rs; i++) tmp[i] = ((int64_t)g.rs_items[i] << 32) | (uint32_t)i;
    qsort(tmp, (size_t)g.n_rs, sizeof(int64_t), cmp64);
    f->n_rowsums = g.n_rs;
    f->rs_items = (int32_t *)malloc(sizeof(int32_t) * (g.n_rs ? g.n_rs : 1));
    f->rs_exact = (int64_t *)malloc(sizeof(int64_t) * (g.n_rs ? g.n_rs : 1));
    f->rs_v32 = (int32_t *)malloc(sizeof(int32_t) * (g.n_rs ? g.n_rs : 1));
    for (int32_t i = 0; i < g.n_rs; i++) {
      int32_t k = (int32_t)(tmp[i] & 0xffffffff);
      f->rs_items[i] = g.rs_items[k];
      f->rs_exact[i] = g.rs_exact[k];
      f->rs_v32[i] = g.rs_v32[k];
    }
    free(tmp);
  }

  /* Rescorer.processWatermark -> updateGlobalItemRowSums, :144-156 (only emitted, non-zero int
   * deltas reach it: RowSumAggregator.java:66) */
  for (int32_t i = 0; i < f->n_rowsums; i++) {
    int32_t d = f->rs_v32[i];
    if (d != 0) {
      s->rowsum_acc += d; /* RowSumProcessWindowRowSum, RowSumAggregator.java:67 */
      int32_t r = global_rowsum_slot(s, f->rs_items[i], 1);
      s->grs_v32[r] = (int32_t)((uint32_t)s->grs_v32[r] + (uint32_t)d);
      s->observed_ref += d; /* :154 */
    }
    int32_t r = global_rowsum_slot(s, f->rs_items[i], 1);
    s->grs_exact[r] += f->rs_exact[i];
  }

  /* Rescorer.scoreItemRows, :158-228 */
  if (s->topk > 0) {
    f->n_topk = f->n_rows;
    f->tk_rows = (int32_t *)malloc(sizeof(int32_t) * (f->n_rows ? f->n_rows : 1));
    f->tk_sizes = (int32_t *)malloc(sizeof(int32_t) * (f->n_rows ? f->n_rows : 1));
    f->tk_values = (int32_t *)malloc(sizeof(int32_t) * ((size_t)f->n_rows * s->topk + 1));
    f->tk_scores = (double *)malloc(sizeof(double) * ((size_t)f->n_rows * s->topk + 1));
  }
  oc_pq *q = s->topk > 0 ? oc_pq_create(s->topk) : NULL;
  for (int32_t i = 0; i < f->n_rows; i++) {
    int32_t item = f->rows[i];
    s->rescored_items++; /* :169 */
    rowmap *gr = global_row(s, item);
    for (int64_t e = f->row_ptr[i]; e < f->row_ptr[i + 1]; e++) /* :172-177 */
      rowmap_add_to(gr, f->cols[e], f->v16[e], f->exact[e]);
    if (!q) continue;
    int32_t item_row_sum = global_rowsum32(s, item); /* :181 */
    oc_pq_reset(q);                                  /* :197 */
    int32_t *slots = rowmap_sorted_slots(gr);
    for (int32_t j = 0; j < gr->n; j++) { /* :199-223 */
      int32_t other = gr->col[slots[j]];
      int16_t count = gr->v16[slots[j]];
      int64_t other_row_sum = global_rowsum32(s, other);
      double score = oc_score_item(count, item_row_sum, other_row_sum, s->observed_ref);
      pq_offer(q, s->topk, other, score);
    }
    free(slots);
    f->tk_rows[i] = item;
    f->tk_sizes[i] = q->size;
    oc_pq_entries(q, f->tk_values + (size_t)i * s->topk, f->tk_scores + (size_t)i * s->topk);
  }
  oc_pq_destroy(q);
  free(order);

  for (int32_t i = 0; i < g.n_rows; i++) rowmap_free(&g.rows[i]);
  free(g.rows);
  i32map_free(&g.row_idx);
  i32map_free(&g.rs_idx);
  free(g.rs_items); free(g.rs_v32); free(g.rs_exact);
}

/* Timer service: fire every pending window whose maxTimestamp <= watermark, ascending. */
EXPORT int32_t oc_process_watermark(oc_state *s, int64_t watermark) {
  int32_t fired = 0;
  if (watermark > s->watermark) s->watermark = watermark;
  for (;;) {
    int32_t best = -1;
    for (int32_t i = 0; i < s->n_pw; i++)
      if (s->pw[i].max_ts <= s->watermark && (best < 0 || s->pw[i].max_ts < s->pw[best].max_ts)) best = i;
    if (best < 0) break;
    pending_window p = s->pw[best];
    s->pw[best] = s->pw[--s->n_pw];
    fire_window(s, &p);
    free(p.users.a);
    free(p.items.a);
    fired++;
  }
  return fired;
}

/* ---- accessors ------------------------------------------------------------------------------ */
EXPORT int32_t oc_n_windows(const oc_state *s) { return s->n_fw; }
EXPORT int64_t oc_window_ts(const oc_state *s, int32_t w) { return s->fw[w].ts; }
EXPORT int32_t oc_window_n_rows(const oc_state *s, int32_t w) { return s->fw[w].n_rows; }
EXPORT int64_t oc_window_nnz(const oc_state *s, int32_t w) { return s->fw[w].row_ptr[s->fw[w].n_rows]; }
EXPORT int64_t oc_window_observed(const oc_state *s, int32_t w) { return s->fw[w].observed_acc; }
EXPORT int32_t oc_window_n_rowsums(const oc_state *s, int32_t w) { return s->fw[w].n_rowsums; }
EXPORT int32_t oc_window_n_topk(const oc_state *s, int32_t w) { return s->fw[w].n_topk; }

EXPORT void oc_window_delta(const oc_state *s, int32_t w, int32_t *rows, int64_t *row_ptr, int32_t *cols,
                            int64_t *exact, int16_t *v16) {
  const fired_window *f = &s->fw[w];
  int64_t nnz = f->row_ptr[f->n_rows];
  if (rows) memcpy(rows, f->rows, sizeof(int32_t) * f->n_rows);
  if (row_ptr) memcpy(row_ptr, f->row_ptr, sizeof(int64_t) * (f->n_rows + 1));
  if (cols) memcpy(cols, f->cols, sizeof(int32_t) * nnz);
  if (exact) memcpy(exact, f->exact, sizeof(int64_t) * nnz);
  if (v16) memcpy(v16, f->v16, sizeof(int16_t) * nnz);
}

EXPORT void oc_window_rowsums(const oc_state *s, int32_t w, int32_t *items, int64_t *exact, int32_t *v32) {
  const fired_window *f = &s->fw[w];
  if (items) memcpy(items, f->rs_items, sizeof(int32_t) * f->n_rowsums);
  if (exact) memcpy(exact, f->rs_exact, sizeof(int64_t) * f->n_rowsums);
  if (v32) memcpy(v32, f->rs_v32, sizeof(int32_t) * f->n_rowsums);
}

EXPORT void oc_window_topk(const oc_state *s, int32_t w, int32_t *rows, int32_t *sizes, int32_t *values,
                           double *scores) {
  const fired_window *f = &s->fw[w];
  if (rows) memcpy(rows, f->tk_rows, sizeof(int32_t) * f->n_topk);
  if (sizes) memcpy(sizes, f->tk_sizes, sizeof(int32_t) * f->n_topk);
  if (values) memcpy(values, f->tk_values, sizeof(int32_t) * (size_t)f->n_topk * s->topk);
  if (scores) memcpy(scores, f->tk_scores, sizeof(double) * (size_t)f->n_topk * s->topk);
}

EXPORT void oc_counters(const oc_state *s, int64_t *out5) {
  out5[0] = s->late_elements;
  out5[1] = s->observed_acc;
  out5[2] = s->rowsum_acc;
  out5[3] = s->rescored_items;
  out5[4] = s->observed_ref;
}

/* Global rows (Rescorer:35 itemRows) as sorted CSR over the items that own a row. */
EXPORT int32_t oc_global_n_rows(const oc_state *s) { return s->n_grows; }
EXPORT int64_t oc_global_nnz(const oc_state *s) {
  int64_t n = 0;
  for (int32_t i = 0; i < s->n_grows; i++) n += s->grows[i].n;
  return n;
}
EXPORT void oc_global_rows(const oc_state *s, int32_t *rows, int64_t *row_ptr, int32_t *cols, int64_t *exact,
                           int16_t *v16) {
  int64_t *tmp = (int64_t *)malloc(sizeof(int64_t) * (s->n_grows ? s->n_grows : 1));
  for (int64_t k = 0; k < s->grow_idx.cap; k++)
    if (s->grow_idx.slot[k] >= 0) tmp[s->grow_idx.slot[k]] = ((int64_t)s->grow_idx.keys[k] << 32) | (uint32_t)s->grow_idx.slot[k];
  qsort(tmp, (size_t)s->n_grows, sizeof(int64_t), cmp64);
  int64_t pos = 0;
  for (int32_t i = 0; i < s->n_grows; i++) {
    const rowmap *r = &s->grows[(int32_t)(tmp[i] & 0xffffffff)];
    rows[i] = (int32_t)(tmp[i] >> 32);
    row_ptr[i] = pos;
    int32_t *slots = rowmap_sorted_slots(r);
    for (int32_t j = 0; j < r->n; j++, pos++) {
      cols[pos] = r->col[slots[j]];
      if (exact) exact[pos] = r->exact[slots[j]];
      if (v16) v16[pos] = r->v16[slots[j]];
    }
    free(slots);
  }
  row_ptr[s->n_grows] = pos;
  free(tmp);
}

/* Global row sums: items with a row-sum entry, the int view (Int2IntOpenHashMap) and exact. */
EXPORT int32_t oc_global_n_rowsums(const oc_state *s) { return s->n_grs; }
EXPORT void oc_global_rowsums(const oc_state *s, int32_t *items, int32_t *v32, int64_t *exact) {
  int64_t *tmp = (int64_t *)malloc(sizeof(int64_t) * (s->n_grs ? s->n_grs : 1));
  for (int64_t k = 0; k < s->grs_idx.cap; k++)
    if (s->grs_idx.slot[k] >= 0) tmp[s->grs_idx.slot[k]] = ((int64_t)s->grs_idx.keys[k] << 32) | (uint32_t)s->grs_idx.slot[k];
  qsort(tmp, (size_t)s->n_grs, sizeof(int64_t), cmp64);
  for (int32_t i = 0; i < s->n_grs; i++) {
    int32_t r = (int32_t)(tmp[i] & 0xffffffff);
    items[i] = (int32_t)(tmp[i] >> 32);
    if (v32) v32[i] = s->grs_v32[r];
    if (exact) exact[i] = s->grs_exact[r];
  }
  free(tmp);
}

/* ------------------------------------------------------------------------------------------ */
/* One-window batch restatement over a CSR of user histories (every user starts empty), the   */
/* shape of the stateless device entry point.  Literal NonSampled:144-151 expansion, exact    */
/* int64 counts, dense accumulator (n_items^2 int64) -- only for small n_items.               */
/* Output: dense counts [n_items*n_items], row sums [n_items], returns observed pairs.        */
/* ------------------------------------------------------------------------------------------ */
EXPORT int64_t oc_batch_dense(int64_t n_users, const int64_t *user_ptr, const int32_t *items, int32_t n_items,
                              int64_t *counts, int64_t *rowsums) {
  int64_t observed = 0;
  memset(counts, 0, sizeof(int64_t) * (size_t)n_items * (size_t)n_items);
  memset(rowsums, 0, sizeof(int64_t) * (size_t)n_items);
  for (int64_t u = 0; u < n_users; u++) {
    const int32_t *h = items + user_ptr[u];
    int64_t n = user_ptr[u + 1] - user_ptr[u];
    for (int64_t q = 0; q < n; q++) { /* new item h[q], history h[0..q) */
      int32_t item = h[q];
      if (q > 0) {
        rowsums[item] += q;
        for (int64_t p = 0; p < q; p++) {
          counts[(int64_t)item * n_items + h[p]] += 1; /* (item, history, +1), :138-139 */
          counts[(int64_t)h[p] * n_items + item] += 1; /* (other, item, +1), :146-147 */
          rowsums[h[p]] += 1;
        }
        observed += 2 * q;
      }
    }
  }
  return observed;
}

/* ------------------------------------------------------------------------------------------ */
/* Multithreaded one-window restatement (bench.py's cpu_baseline; BASELINE.md: "CPU restatement, */
/* not the JVM reference").  The job's keyed data-parallelism with threads for subtasks: thread t  */
/* owns the rows a with a mod n_threads == t (keyBy(ItemCooccurrences::getItem),                  */
/* FlinkCooccurrences.java:152) and expands every user's window record by record                 */
/* (NonSampled:129-161, empty histories), keeping the (row, other) increments of its own rows in  */
/* Int2ShortOpenHashMap restatements (ItemRowAggregator.java:26-31).  Returns the distinct keys;  */
/* *pairs = the ordered pairs seen (each counted once, by its row's owner).                      */
/* ------------------------------------------------------------------------------------------ */
#include <pthread.h>

typedef struct {
  int64_t n_users;
  const int64_t *user_ptr;
  const int32_t *items;
  int32_t n_items, n_threads, t;
  int64_t nnz, pairs;
  uint64_t *row_cs;  /* optional per-row outputs (oc_row_key_hash below) */
  int64_t *row_nnz, *row_sum;
} mt_job;

/* Row checksum entry hash (the same definition as the library's cooc_verify_batch, include/cooc.h):
 * splitmix64 of (column << 32 | exact count); a row's checksum is the sum of its entries' hashes
 * mod 2^64, so it does not depend on the order the row's keys are visited in. */
static uint64_t oc_row_key_hash(int32_t col, uint64_t count) {
  uint64_t x = ((uint64_t)(uint32_t)col << 32) ^ count;
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

static void *mt_run(void *arg) {
  mt_job *j = (mt_job *)arg;
  const int32_t T = j->n_threads, t = j->t;
  const int32_t n_own = (j->n_items - t + T - 1) / T;
  rowmap *rows = (rowmap *)calloc((size_t)(n_own > 0 ? n_own : 1), sizeof(rowmap));
  char *live = (char *)calloc((size_t)(n_own > 0 ? n_own : 1), 1);
  int64_t pairs = 0;
  for (int64_t u = 0; u < j->n_users; u++) {
    const int32_t *h = j->items + j->user_ptr[u];
    const int64_t n = j->user_ptr[u + 1] - j->user_ptr[u];
    for (int64_t p = 1; p < n; p++) { /* item x = h[p] against its history h[0..p) */
      const int32_t x = h[p];
      for (int64_t q = 0; q < p; q++) {
        const int32_t o = h[q];
        if (x % T == t) { /* record (x, history, +1), NonSampled:138-139 */
          rowmap *r = &rows[x / T];
          if (!live[x / T]) { rowmap_init(r); live[x / T] = 1; }
          rowmap_add_to(r, o, 1, 1);
          pairs++;
        }
        if (o % T == t) { /* record (o, x, +1), NonSampled:144-147 */
          rowmap *r = &rows[o / T];
          if (!live[o / T]) { rowmap_init(r); live[o / T] = 1; }
          rowmap_add_to(r, x, 1, 1);
          pairs++;
        }
      }
    }
  }
  int64_t nnz = 0;
  for (int32_t i = 0; i < n_own; i++) {
    if (j->row_cs) { /* row a = i * T + t (rows without keys stay 0) */
      const int64_t a = (int64_t)i * T + t;
      uint64_t cs = 0;
      int64_t sum = 0;
      if (live[i])
        for (int32_t e = 0; e < rows[i].n; e++) {
          cs += oc_row_key_hash(rows[i].col[e], (uint64_t)rows[i].exact[e]);
          sum += rows[i].exact[e];
        }
      j->row_cs[a] = cs;
      j->row_nnz[a] = live[i] ? rows[i].n : 0;
      j->row_sum[a] = sum;
    }
    if (live[i]) { nnz += rows[i].n; rowmap_free(&rows[i]); }
  }
  free(rows);
  free(live);
  j->nnz = nnz;
  j->pairs = pairs;
  return NULL;
}

/* The restatement above, with optional per-row outputs: checksum (sum of oc_row_key_hash over the
 * row's keys), distinct keys and the sum of the exact counts (int64 [n_items] each, or all NULL). */
EXPORT int64_t oc_count_batch_mt_rows(int64_t n_users, const int64_t *user_ptr, const int32_t *items, int32_t n_items,
                                      int32_t n_threads, int64_t *pairs, uint64_t *row_cs, int64_t *row_nnz,
                                      int64_t *row_sum) {
  if (n_threads < 1) n_threads = 1;
  mt_job *jobs = (mt_job *)calloc((size_t)n_threads, sizeof(mt_job));
  pthread_t *th = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
  for (int32_t t = 0; t < n_threads; t++) {
    jobs[t] = (mt_job){n_users, user_ptr, items, n_items, n_threads, t, 0, 0, row_cs, row_nnz, row_sum};
    pthread_create(&th[t], NULL, mt_run, &jobs[t]);
  }
  int64_t nnz = 0, pr = 0;
  for (int32_t t = 0; t < n_threads; t++) {
    pthread_join(th[t], NULL);
    nnz += jobs[t].nnz;
    pr += jobs[t].pairs;
  }
  free(jobs);
  free(th);
  if (pairs) *pairs = pr;
  return nnz;
}

EXPORT int64_t oc_count_batch_mt(int64_t n_users, const int64_t *user_ptr, const int32_t *items, int32_t n_items,
                                 int32_t n_threads, int64_t *pairs) {
  return oc_count_batch_mt_rows(n_users, user_ptr, items, n_items, n_threads, pairs, NULL, NULL, NULL);
}

/* ------------------------------------------------------------------------------------------ */
/* Per-row checksums in closed form, for exactness checks at the benchmark's size (1e10 pairs).  */
/* Row a of C = A^T A - diag(colsum A) (the sum over windows of NonSampled:113-165, SURVEY.md     */
/* §0.3) is the sum of the lists of the users holding a (once per occurrence of a), minus one at  */
/* column a per occurrence.  Gustavson row by row: the users of every item by a counting sort     */
/* (the transpose of A), then a dense int64 accumulator per thread and a touched-column list.     */
/* Rows are handed out in blocks of 64 from an atomic counter.  Writes the same per-row checksum, */
/* key count and count sum as oc_count_batch_mt_rows (it is cross-checked against it and against */
/* scipy in tests/test_oracle_semantics.py).  Returns the distinct keys; *pairs = ordered pairs.  */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  const int64_t *user_ptr;
  const int32_t *items;
  const int64_t *item_ptr; /* [n_items + 1] */
  const int64_t *item_users;
  int32_t n_items;
  int64_t *next;           /* shared row-block counter */
  uint64_t *row_cs;
  int64_t *row_nnz, *row_sum;
  int64_t nnz, pairs;
} gus_job;

static void *gus_run(void *arg) {
  gus_job *j = (gus_job *)arg;
  const int32_t M = j->n_items;
  int64_t *acc = (int64_t *)calloc((size_t)M, sizeof(int64_t));
  int32_t *touched = (int32_t *)malloc(sizeof(int32_t) * (size_t)M);
  int64_t nnz = 0, pairs = 0;
  for (;;) {
    const int64_t b0 = __atomic_fetch_add(j->next, 64, __ATOMIC_RELAXED);
    if (b0 >= M) break;
    const int64_t b1 = b0 + 64 < M ? b0 + 64 : M;
    for (int64_t a = b0; a < b1; a++) {
      int32_t nt = 0;
      for (int64_t k = j->item_ptr[a]; k < j->item_ptr[a + 1]; k++) {
        const int64_t u = j->item_users[k];
        for (int64_t p = j->user_ptr[u]; p < j->user_ptr[u + 1]; p++) {
          const int32_t b = j->items[p];
          if (acc[b]++ == 0) touched[nt++] = b;
        }
      }
      const int64_t occ = j->item_ptr[a + 1] - j->item_ptr[a];
      acc[a] -= occ; /* the pair of a position with itself */
      uint64_t cs = 0;
      int64_t n = 0, sum = 0;
      for (int32_t i = 0; i < nt; i++) {
        const int32_t b = touched[i];
        if (acc[b]) {
          cs += oc_row_key_hash(b, (uint64_t)acc[b]);
          n++;
          sum += acc[b];
        }
        acc[b] = 0;
      }
      j->row_cs[a] = cs;
      j->row_nnz[a] = n;
      j->row_sum[a] = sum;
      nnz += n;
      pairs += sum;
    }
  }
  free(acc);
  free(touched);
  j->nnz = nnz;
  j->pairs = pairs;
  return NULL;
}

EXPORT int64_t oc_row_checksums(int64_t n_users, const int64_t *user_ptr, const int32_t *items, int32_t n_items,
                                int32_t n_threads, int64_t *pairs, uint64_t *row_cs, int64_t *row_nnz,
                                int64_t *row_sum) {
  if (n_threads < 1) n_threads = 1;
  const int64_t n = n_users > 0 ? user_ptr[n_users] : 0;
  int64_t *item_ptr = (int64_t *)calloc((size_t)n_items + 1, sizeof(int64_t));
  int64_t *item_users = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  for (int64_t p = 0; p < n; p++) item_ptr[items[p] + 1]++;
  for (int32_t a = 0; a < n_items; a++) item_ptr[a + 1] += item_ptr[a];
  int64_t *cur = (int64_t *)malloc(sizeof(int64_t) * (size_t)n_items);
  memcpy(cur, item_ptr, sizeof(int64_t) * (size_t)n_items);
  for (int64_t u = 0; u < n_users; u++)
    for (int64_t p = user_ptr[u]; p < user_ptr[u + 1]; p++) item_users[cur[items[p]]++] = u;
  free(cur);
  int64_t next = 0;
  gus_job *jobs = (gus_job *)calloc((size_t)n_threads, sizeof(gus_job));
  pthread_t *th = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
  for (int32_t t = 0; t < n_threads; t++) {
    jobs[t] = (gus_job){user_ptr, items, item_ptr, item_users, n_items, &next, row_cs, row_nnz, row_sum, 0, 0};
    pthread_create(&th[t], NULL, gus_run, &jobs[t]);
  }
  int64_t nnz = 0, pr = 0;
  for (int32_t t = 0; t < n_threads; t++) {
    pthread_join(th[t], NULL);
    nnz += jobs[t].nnz;
    pr += jobs[t].pairs;
  }
  free(jobs);
  free(th);
  free(item_ptr);
  free(item_users);
  if (pairs) *pairs = pr;
  return nnz;
}

/* ------------------------------------------------------------------------------------------ */
/* The rescorer's top-k loop over given rows (ItemRowRescorerTwoInputStreamOperator.java:195-223, */
/* scoreItem :230-241, IntDoublePriorityQueue add/update :132-150), each row's entries fed in the */
/* order given (a device row's own order: the tie order).  Row j is item row_items[j] with entries */
/* [row_ptr[j], row_ptr[j + 1]) of cols / cnt16 (the Int2ShortOpenHashMap values); rs32 holds every */
/* item's int row sum (Int2IntOpenHashMap.get, 0 when absent) and observed the rescorer's long.    */
/* Rows are dealt to n_threads threads.  Heaps out as sizes[n_rows], values / scores[n_rows * k],  */
/* positions 1..size (iterator(), IntDoublePriorityQueue.java:215-242).                            */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  int64_t n_rows, j0, j1;
  const int32_t *row_items;
  const int64_t *row_ptr;
  const int32_t *cols;
  const int16_t *cnt16;
  const int32_t *rs32;
  int64_t observed;
  int32_t k;
  int32_t *sizes, *values;
  double *scores;
} topk_job;

static void *topk_run(void *arg) {
  topk_job *j = (topk_job *)arg;
  oc_pq *q = oc_pq_create(j->k);
  for (int64_t r = j->j0; r < j->j1; r++) {
    oc_pq_reset(q);
    const int32_t a = j->row_items[r];
    for (int64_t e = j->row_ptr[r]; e < j->row_ptr[r + 1]; e++) {
      const int32_t b = j->cols[e];
      pq_offer(q, j->k, b, oc_score_item(j->cnt16[e], j->rs32[a], j->rs32[b], j->observed));
    }
    j->sizes[r] = q->size;
    oc_pq_entries(q, j->values + r * j->k, j->scores + r * j->k);
  }
  oc_pq_destroy(q);
  return NULL;
}

EXPORT void oc_rows_topk(int64_t n_rows, const int32_t *row_items, const int64_t *row_ptr, const int32_t *cols,
                         const int16_t *cnt16, const int32_t *rs32, int64_t observed, int32_t k, int32_t n_threads,
                         int32_t *sizes, int32_t *values, double *scores) {
  if (n_threads < 1) n_threads = 1;
  topk_job *jobs = (topk_job *)calloc((size_t)n_threads, sizeof(topk_job));
  pthread_t *th = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
  for (int32_t t = 0; t < n_threads; t++) {
    jobs[t] = (topk_job){n_rows, n_rows * t / n_threads, n_rows * (t + 1) / n_threads, row_items, row_ptr, cols,
                         cnt16, rs32, observed, k, sizes, values, scores};
    pthread_create(&th[t], NULL, topk_run, &jobs[t]);
  }
  for (int32_t t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
}
