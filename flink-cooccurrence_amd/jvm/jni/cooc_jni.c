/* cooc_jni.c -- JNI shim of com.github.uce.flinkcooccurrences.CoocNative over include/cooc.h.
 *
 * Build (a JDK 8 is needed; there is none in the build container, so this file is uncompiled here):
 *   gcc -O2 -shared -fPIC -I"$JAVA_HOME/include" -I"$JAVA_HOME/include/linux" -I../../../include \
 *       cooc_jni.c -L../csrc -lcooc_hip -Wl,-rpath,'$ORIGIN' -o libcooc_jni.so
 * (jvm/Makefile).  Error behaviour: COOC_ERR_ARG -> IllegalArgumentException, any other non-zero
 * status -> IllegalStateException, message = cooc_last_error(handle), as the reference throws
 * (ItemRowRescorerTwoInputStreamOperator.java:52-54,72-79,91-93); a failed native allocation ->
 * OutOfMemoryError.
 *
 * Java arrays are never pinned across a library call: the calls stage data, launch kernels and
 * synchronise the GPU, and a JNI critical region around them would stall the garbage collector of
 * every subtask sharing the TaskManager JVM.  Inputs are copied out of the Java heap with
 * Get<Type>ArrayRegion into native scratch, outputs land in native scratch and are copied back with
 * Set<Type>ArrayRegion after the call.  No caller pointer is kept (cooc.h ownership rules). */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "cooc.h"

#define H(h) ((cooc_ctx *)(intptr_t)(h))

static void throw_class(JNIEnv *env, const char *cls, const char *msg) {
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, msg);
}

static void throw_status(JNIEnv *env, const cooc_ctx *ctx, int st) {
  throw_class(env, st == COOC_ERR_ARG ? "java/lang/IllegalArgumentException" : "java/lang/IllegalStateException",
              cooc_last_error(ctx));
}

static int check(JNIEnv *env, const cooc_ctx *ctx, int st) {
  if (st) throw_status(env, ctx, st);
  return st;
}

/* Native scratch for one Java array argument: n elements of elem bytes (a NULL array -> NULL). */
typedef struct {
  jarray a;
  jsize n;
  void *p;
} scratch;

/* Allocates the scratch of array a (its length, or want elements when want >= 0); copy_in: fill it
 * from the array.  Returns 0, or -1 with an exception pending. */
static int scratch_get(JNIEnv *env, scratch *s, jarray a, size_t elem, jsize want, int copy_in, char type) {
  s->a = a;
  s->p = NULL;
  s->n = 0;
  if (!a) return 0;
  const jsize len = (*env)->GetArrayLength(env, a);
  s->n = want >= 0 ? want : len;
  if (s->n > len) {
    throw_class(env, "java/lang/ArrayIndexOutOfBoundsException", "array shorter than the native call needs");
    return -1;
  }
  s->p = malloc(elem * (size_t)(s->n > 0 ? s->n : 1));
  if (!s->p) {
    throw_class(env, "java/lang/OutOfMemoryError", "cooc_jni: native scratch allocation failed");
    return -1;
  }
  if (copy_in && s->n > 0) {
    switch (type) {
      case 'I': (*env)->GetIntArrayRegion(env, (jintArray)a, 0, s->n, (jint *)s->p); break;
      case 'J': (*env)->GetLongArrayRegion(env, (jlongArray)a, 0, s->n, (jlong *)s->p); break;
      case 'S': (*env)->GetShortArrayRegion(env, (jshortArray)a, 0, s->n, (jshort *)s->p); break;
      case 'D': (*env)->GetDoubleArrayRegion(env, (jdoubleArray)a, 0, s->n, (jdouble *)s->p); break;
    }
    if ((*env)->ExceptionCheck(env)) return -1;
  }
  return 0;
}

/* Copies the scratch back into its array (n elements) and frees it. */
static void scratch_put(JNIEnv *env, scratch *s, int copy_out, char type, jsize n) {
  if (s->a && s->p && copy_out && n > 0 && !(*env)->ExceptionCheck(env)) {
    switch (type) {
      case 'I': (*env)->SetIntArrayRegion(env, (jintArray)s->a, 0, n, (const jint *)s->p); break;
      case 'J': (*env)->SetLongArrayRegion(env, (jlongArray)s->a, 0, n, (const jlong *)s->p); break;
      case 'S': (*env)->SetShortArrayRegion(env, (jshortArray)s->a, 0, n, (const jshort *)s->p); break;
      case 'D': (*env)->SetDoubleArrayRegion(env, (jdoubleArray)s->a, 0, n, (const jdouble *)s->p); break;
    }
  }
  free(s->p);
  s->p = NULL;
}

JNIEXPORT jlong JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_create(
    JNIEnv *env, jclass cls, jintArray devices, jint subtask, jint nItems, jint topK, jint flags, jlong windowMs,
    jshort userCut) {
  cooc_config cfg = {-1, nItems, topK, flags, windowMs, userCut, 0}; /* userCut 0 = the non-sampled path */
  cooc_ctx *h = NULL;
  scratch d;
  if (scratch_get(env, &d, devices, sizeof(jint), -1, 1, 'I')) {
    scratch_put(env, &d, 0, 'I', 0);
    return 0;
  }
  const int st = d.n ? cooc_create_on(&cfg, (const int32_t *)d.p, d.n, subtask, &h) : cooc_create(&cfg, &h);
  scratch_put(env, &d, 0, 'I', 0);
  if (check(env, NULL, st)) return 0;
  return (jlong)(intptr_t)h;
}

JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_destroy(JNIEnv *env, jclass cls, jlong h) {
  cooc_destroy(H(h));
}

JNIEXPORT jlong JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_processElements(
    JNIEnv *env, jclass cls, jlong h, jint n, jintArray users, jintArray items, jlongArray ts) {
  int64_t late = 0;
  scratch u, i, t;
  u.p = i.p = t.p = NULL;
  if (!scratch_get(env, &u, users, sizeof(jint), n, 1, 'I') && !scratch_get(env, &i, items, sizeof(jint), n, 1, 'I') &&
      !scratch_get(env, &t, ts, sizeof(jlong), n, 1, 'J')) {
    check(env, H(h), cooc_op_process_elements(H(h), n, (const int32_t *)u.p, (const int32_t *)i.p,
                                              (const int64_t *)t.p, &late));
  }
  scratch_put(env, &t, 0, 'J', 0);
  scratch_put(env, &i, 0, 'I', 0);
  scratch_put(env, &u, 0, 'I', 0);
  return late;
}

JNIEXPORT jboolean JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_processWatermark(
    JNIEnv *env, jclass cls, jlong h, jlong watermark, jlongArray info) {
  int32_t fired = 0;
  cooc_window_info wi;
  if (check(env, H(h), cooc_op_process_watermark(H(h), watermark, &fired, &wi)) || !fired) return JNI_FALSE;
  const jlong v[6] = {wi.ts, wi.nnz, wi.observed, wi.n_rows, wi.topk, wi.n_topk};
  (*env)->SetLongArrayRegion(env, info, 0, 6, v);
  return JNI_TRUE;
}

/* The fired window's delta rows and their starts: rows int[nRows], rowPtr long[nRows + 1] (entry
 * offsets; the entries themselves stream out with copyDeltaRange). */
JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_copyDeltaRows(
    JNIEnv *env, jclass cls, jlong h, jintArray rows, jlongArray rowPtr) {
  scratch r, p;
  r.p = p.p = NULL;
  const jsize n = rows ? (*env)->GetArrayLength(env, rows) : 0;
  if (!scratch_get(env, &r, rows, sizeof(jint), n, 0, 'I') && !scratch_get(env, &p, rowPtr, sizeof(jlong), n + 1, 0, 'J'))
    check(env, H(h), cooc_copy_window_delta(H(h), (int32_t *)r.p, (int64_t *)p.p, NULL, NULL, NULL));
  scratch_put(env, &p, 1, 'J', n + 1);
  scratch_put(env, &r, 1, 'I', n);
}

/* Entries of delta rows [rowBegin, rowEnd): cols int[n], cnt16 short[n] with n = rowPtr[rowEnd] -
 * rowPtr[rowBegin] (the caller sizes ranges so that n fits a Java array). */
JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_copyDeltaRange(
    JNIEnv *env, jclass cls, jlong h, jint rowBegin, jint rowEnd, jint n, jintArray cols, jshortArray cnt16) {
  scratch c, v;
  c.p = v.p = NULL;
  if (!scratch_get(env, &c, cols, sizeof(jint), n, 0, 'I') && !scratch_get(env, &v, cnt16, sizeof(jshort), n, 0, 'S'))
    check(env, H(h), cooc_copy_window_delta_range(H(h), rowBegin, rowEnd, (int64_t)n, (int32_t *)c.p, NULL,
                                                  (int16_t *)v.p));
  scratch_put(env, &v, 1, 'S', n);
  scratch_put(env, &c, 1, 'I', n);
}

JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_copyRowSums(
    JNIEnv *env, jclass cls, jlong h, jintArray items, jintArray delta32) {
  scratch i, d;
  i.p = d.p = NULL;
  const jsize n = items ? (*env)->GetArrayLength(env, items) : 0;
  if (!scratch_get(env, &i, items, sizeof(jint), n, 0, 'I') && !scratch_get(env, &d, delta32, sizeof(jint), n, 0, 'I'))
    check(env, H(h), cooc_copy_window_rowsums(H(h), (int32_t *)i.p, NULL, (int32_t *)d.p));
  scratch_put(env, &d, 1, 'I', n);
  scratch_put(env, &i, 1, 'I', n);
}

JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_copyTopK(
    JNIEnv *env, jclass cls, jlong h, jintArray rows, jintArray sizes, jintArray values, jdoubleArray scores) {
  scratch r, z, v, s;
  r.p = z.p = v.p = s.p = NULL;
  const jsize n = rows ? (*env)->GetArrayLength(env, rows) : 0;
  const jsize nv = values ? (*env)->GetArrayLength(env, values) : 0;
  if (!scratch_get(env, &r, rows, sizeof(jint), n, 0, 'I') && !scratch_get(env, &z, sizes, sizeof(jint), n, 0, 'I') &&
      !scratch_get(env, &v, values, sizeof(jint), nv, 0, 'I') &&
      !scratch_get(env, &s, scores, sizeof(jdouble), nv, 0, 'D'))
    check(env, H(h), cooc_copy_window_topk(H(h), (int32_t *)r.p, (int32_t *)z.p, (int32_t *)v.p, (double *)s.p));
  scratch_put(env, &s, 1, 'D', nv);
  scratch_put(env, &v, 1, 'I', nv);
  scratch_put(env, &z, 1, 'I', n);
  scratch_put(env, &r, 1, 'I', n);
}

JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_counters(JNIEnv *env, jclass cls, jlong h,
                                                                                  jlongArray out5) {
  int64_t c[5] = {0, 0, 0, 0, 0};
  if (check(env, H(h), cooc_op_counters(H(h), c))) return;
  const jlong v[5] = {c[0], c[1], c[2], c[3], c[4]};
  (*env)->SetLongArrayRegion(env, out5, 0, 5, v);
}

JNIEXPORT jlongArray JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_countBatch(
    JNIEnv *env, jclass cls, jlong h, jlongArray userPtr, jintArray items) {
  const jsize n_users = (*env)->GetArrayLength(env, userPtr) - 1;
  cooc_window_info wi;
  scratch p, i;
  p.p = i.p = NULL;
  int st = -1;
  if (!scratch_get(env, &p, userPtr, sizeof(jlong), -1, 1, 'J') && !scratch_get(env, &i, items, sizeof(jint), -1, 1, 'I'))
    st = check(env, H(h), cooc_count_host(H(h), n_users, (const int64_t *)p.p, (const int32_t *)i.p, &wi));
  scratch_put(env, &i, 0, 'I', 0);
  scratch_put(env, &p, 0, 'J', 0);
  if (st) return NULL;
  jlongArray out = (*env)->NewLongArray(env, 2);
  if (out) {
    const jlong v[2] = {wi.nnz, wi.observed};
    (*env)->SetLongArrayRegion(env, out, 0, 2, v);
  }
  return out;
}

/* ---- multi-GPU (p > 1, one window): the exchange inside the library over RCCL ---- */
JNIEXPORT jbyteArray JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_commUniqueId(JNIEnv *env, jclass cls) {
  uint8_t id[COOC_COMM_ID_BYTES];
  if (check(env, NULL, cooc_comm_unique_id(id))) return NULL;
  jbyteArray out = (*env)->NewByteArray(env, COOC_COMM_ID_BYTES);
  if (out) (*env)->SetByteArrayRegion(env, out, 0, COOC_COMM_ID_BYTES, (const jbyte *)id);
  return out;
}

JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_commInit(
    JNIEnv *env, jclass cls, jlong h, jbyteArray id, jint rank, jint world) {
  uint8_t buf[COOC_COMM_ID_BYTES];
  if (!id || (*env)->GetArrayLength(env, id) != COOC_COMM_ID_BYTES) {
    throw_class(env, "java/lang/IllegalArgumentException", "the communicator id is COOC_COMM_ID_BYTES bytes");
    return;
  }
  (*env)->GetByteArrayRegion(env, id, 0, COOC_COMM_ID_BYTES, (jbyte *)buf);
  check(env, H(h), cooc_comm_init(H(h), buf, rank, world));
}

JNIEXPORT jlongArray JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_countOwned(
    JNIEnv *env, jclass cls, jlong h, jlongArray userPtr, jintArray items) {
  const jsize n_users = (*env)->GetArrayLength(env, userPtr) - 1;
  cooc_owned_info oi;
  cooc_window_info wi;
  scratch p, i;
  p.p = i.p = NULL;
  int st = -1;
  if (!scratch_get(env, &p, userPtr, sizeof(jlong), -1, 1, 'J') && !scratch_get(env, &i, items, sizeof(jint), -1, 1, 'I'))
    st = check(env, H(h), cooc_count_owned_host(H(h), n_users, (const int64_t *)p.p, (const int32_t *)i.p, &oi, &wi));
  scratch_put(env, &i, 0, 'I', 0);
  scratch_put(env, &p, 0, 'J', 0);
  if (st) return NULL;
  jlongArray out = (*env)->NewLongArray(env, 4);
  if (out) {
    const jlong v[4] = {wi.nnz, wi.observed, wi.n_rows, oi.observed};
    (*env)->SetLongArrayRegion(env, out, 0, 4, v);
  }
  return out;
}

JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_copyBatch(
    JNIEnv *env, jclass cls, jlong h, jlongArray rowPtr, jintArray cols, jshortArray cnt16, jintArray rowSums32) {
  scratch p, c, v, r;
  p.p = c.p = v.p = r.p = NULL;
  if (!scratch_get(env, &p, rowPtr, sizeof(jlong), -1, 0, 'J') && !scratch_get(env, &c, cols, sizeof(jint), -1, 0, 'I') &&
      !scratch_get(env, &v, cnt16, sizeof(jshort), -1, 0, 'S') &&
      !scratch_get(env, &r, rowSums32, sizeof(jint), -1, 0, 'I'))
    check(env, H(h), cooc_copy_batch(H(h), (int64_t *)p.p, (int32_t *)c.p, NULL, (int16_t *)v.p, NULL, (int32_t *)r.p));
  scratch_put(env, &r, 1, 'I', r.n);
  scratch_put(env, &v, 1, 'S', v.n);
  scratch_put(env, &c, 1, 'I', c.n);
  scratch_put(env, &p, 1, 'J', p.n);
}

JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_topKItems(
    JNIEnv *env, jclass cls, jlong h, jint k, jint flags, jintArray items, jintArray sizes, jintArray values,
    jdoubleArray scores) {
  scratch i, z, v, s;
  i.p = z.p = v.p = s.p = NULL;
  const jsize n = items ? (*env)->GetArrayLength(env, items) : 0;
  if (!scratch_get(env, &i, items, sizeof(jint), n, 1, 'I') && !scratch_get(env, &z, sizes, sizeof(jint), n, 0, 'I') &&
      !scratch_get(env, &v, values, sizeof(jint), n * k, 0, 'I') &&
      !scratch_get(env, &s, scores, sizeof(jdouble), n * k, 0, 'D'))
    check(env, H(h), cooc_topk_items(H(h), k, flags, n, (const int32_t *)i.p, (int32_t *)z.p, (int32_t *)v.p,
                                     (double *)s.p));
  scratch_put(env, &s, 1, 'D', n * k);
  scratch_put(env, &v, 1, 'I', n * k);
  scratch_put(env, &z, 1, 'I', n);
  scratch_put(env, &i, 0, 'I', 0);
}

/* ---- owned rows / heaps in row ranges (C-ABI 6): a C3 share never fits one Java array ---- */
JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_copyBatchRange(
    JNIEnv *env, jclass cls, jlong h, jint rowBegin, jint rowEnd, jint n, jintArray cols, jshortArray cnt16) {
  scratch c, v;
  c.p = v.p = NULL;
  if (!scratch_get(env, &c, cols, sizeof(jint), n, 0, 'I') && !scratch_get(env, &v, cnt16, sizeof(jshort), n, 0, 'S'))
    check(env, H(h), cooc_copy_batch_range(H(h), rowBegin, rowEnd, n, (int32_t *)c.p, NULL, (int16_t *)v.p));
  scratch_put(env, &v, 1, 'S', n);
  scratch_put(env, &c, 1, 'I', n);
}

JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_topKOwned(
    JNIEnv *env, jclass cls, jlong h, jint k, jint flags) {
  check(env, H(h), cooc_topk_owned_host(H(h), k, flags));
}

JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_copyTopKRange(
    JNIEnv *env, jclass cls, jlong h, jint rowBegin, jint rowEnd, jint k, jintArray sizes, jintArray values,
    jdoubleArray scores) {
  const jsize n = rowEnd - rowBegin;
  scratch z, v, s;
  z.p = v.p = s.p = NULL;
  if (!scratch_get(env, &z, sizes, sizeof(jint), n, 0, 'I') && !scratch_get(env, &v, values, sizeof(jint), n * k, 0, 'I') &&
      !scratch_get(env, &s, scores, sizeof(jdouble), n * k, 0, 'D'))
    check(env, H(h), cooc_copy_topk_batch_range(H(h), rowBegin, rowEnd, k, (int32_t *)z.p, (int32_t *)v.p, (double *)s.p));
  scratch_put(env, &s, 1, 'D', n * k);
  scratch_put(env, &v, 1, 'I', n * k);
  scratch_put(env, &z, 1, 'I', n);
}

JNIEXPORT jlongArray JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_commAllGather(
    JNIEnv *env, jclass cls, jlong h, jlong value, jint world) {
  jlong *buf = (jlong *)malloc(sizeof(jlong) * (size_t)(world > 0 ? world : 1));
  if (!buf) {
    throw_class(env, "java/lang/OutOfMemoryError", "cooc_jni: native scratch allocation failed");
    return NULL;
  }
  jlongArray out = NULL;
  if (!check(env, H(h), cooc_comm_allgather_i64(H(h), value, (int64_t *)buf))) {
    out = (*env)->NewLongArray(env, world);
    if (out) (*env)->SetLongArrayRegion(env, out, 0, world, buf);
  }
  free(buf);
  return out;
}
