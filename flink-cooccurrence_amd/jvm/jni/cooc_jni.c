/* cooc_jni.c -- JNI shim of com.github.uce.flinkcooccurrences.CoocNative over include/cooc.h.
 *
 * Build (a JDK 8 is needed; there is none in the build container, so this file is uncompiled here):
 *   gcc -O2 -shared -fPIC -I"$JAVA_HOME/include" -I"$JAVA_HOME/include/linux" -I../../../include \
 *       cooc_jni.c -L../csrc -lcooc_hip -Wl,-rpath,'$ORIGIN' -o libcooc_jni.so
 * (jvm/Makefile).  Error behaviour: COOC_ERR_ARG -> IllegalArgumentException, any other non-zero
 * status -> IllegalStateException, message = cooc_last_error(handle), as the reference throws
 * (ItemRowRescorerTwoInputStreamOperator.java:52-54,72-79,91-93).  Arrays are pinned with
 * Get/ReleasePrimitiveArrayCritical around one C call each; no caller pointer is kept (cooc.h
 * ownership rules). */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "cooc.h"

#define H(h) ((cooc_ctx *)(intptr_t)(h))

static void throw_status(JNIEnv *env, const cooc_ctx *ctx, int st) {
  const char *cls = st == COOC_ERR_ARG ? "java/lang/IllegalArgumentException" : "java/lang/IllegalStateException";
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, cooc_last_error(ctx));
}

static int check(JNIEnv *env, const cooc_ctx *ctx, int st) {
  if (st) throw_status(env, ctx, st);
  return st;
}

/* A pinned primitive array (NULL array -> NULL pointer). */
typedef struct {
  jarray a;
  void *p;
} pin;

static pin pin_get(JNIEnv *env, jarray a) {
  pin x = {a, NULL};
  if (a) x.p = (*env)->GetPrimitiveArrayCritical(env, a, NULL);
  return x;
}

static void pin_put(JNIEnv *env, pin x, int copy_back) {
  if (x.a && x.p) (*env)->ReleasePrimitiveArrayCritical(env, x.a, x.p, copy_back ? 0 : JNI_ABORT);
}

JNIEXPORT jlong JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_create(
    JNIEnv *env, jclass cls, jintArray devices, jint subtask, jint nItems, jint topK, jint flags, jlong windowMs,
    jshort userCut) {
  cooc_config cfg = {-1, nItems, topK, flags, windowMs, userCut, 0}; /* userCut 0 = the non-sampled path */
  cooc_ctx *h = NULL;
  const jsize n = devices ? (*env)->GetArrayLength(env, devices) : 0;
  jint *d = n ? (*env)->GetIntArrayElements(env, devices, NULL) : NULL;
  int st = n ? cooc_create_on(&cfg, (const int32_t *)d, n, subtask, &h) : cooc_create(&cfg, &h);
  if (d) (*env)->ReleaseIntArrayElements(env, devices, d, JNI_ABORT);
  if (check(env, NULL, st)) return 0;
  return (jlong)(intptr_t)h;
}

JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_destroy(JNIEnv *env, jclass cls, jlong h) {
  cooc_destroy(H(h));
}

JNIEXPORT jlong JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_processElements(
    JNIEnv *env, jclass cls, jlong h, jint n, jintArray users, jintArray items, jlongArray ts) {
  int64_t late = 0;
  pin u = pin_get(env, users), i = pin_get(env, items), t = pin_get(env, ts);
  const int st = cooc_op_process_elements(H(h), n, (const int32_t *)u.p, (const int32_t *)i.p,
                                          (const int64_t *)t.p, &late);
  pin_put(env, t, 0);
  pin_put(env, i, 0);
  pin_put(env, u, 0);
  check(env, H(h), st);
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

JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_copyDelta(
    JNIEnv *env, jclass cls, jlong h, jintArray rows, jlongArray rowPtr, jintArray cols, jshortArray cnt16) {
  pin r = pin_get(env, rows), p = pin_get(env, rowPtr), c = pin_get(env, cols), v = pin_get(env, cnt16);
  const int st = cooc_copy_window_delta(H(h), (int32_t *)r.p, (int64_t *)p.p, (int32_t *)c.p, NULL, (int16_t *)v.p);
  pin_put(env, v, 1);
  pin_put(env, c, 1);
  pin_put(env, p, 1);
  pin_put(env, r, 1);
  check(env, H(h), st);
}

JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_copyRowSums(
    JNIEnv *env, jclass cls, jlong h, jintArray items, jintArray delta32) {
  pin i = pin_get(env, items), d = pin_get(env, delta32);
  const int st = cooc_copy_window_rowsums(H(h), (int32_t *)i.p, NULL, (int32_t *)d.p);
  pin_put(env, d, 1);
  pin_put(env, i, 1);
  check(env, H(h), st);
}

JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_copyTopK(
    JNIEnv *env, jclass cls, jlong h, jintArray rows, jintArray sizes, jintArray values, jdoubleArray scores) {
  pin r = pin_get(env, rows), z = pin_get(env, sizes), v = pin_get(env, values), s = pin_get(env, scores);
  const int st = cooc_copy_window_topk(H(h), (int32_t *)r.p, (int32_t *)z.p, (int32_t *)v.p, (double *)s.p);
  pin_put(env, s, 1);
  pin_put(env, v, 1);
  pin_put(env, z, 1);
  pin_put(env, r, 1);
  check(env, H(h), st);
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
  pin p = pin_get(env, userPtr), i = pin_get(env, items);
  const int st = cooc_count_host(H(h), n_users, (const int64_t *)p.p, (const int32_t *)i.p, &wi);
  pin_put(env, i, 0);
  pin_put(env, p, 0);
  if (check(env, H(h), st)) return NULL;
  jlongArray out = (*env)->NewLongArray(env, 2);
  if (out) {
    const jlong v[2] = {wi.nnz, wi.observed};
    (*env)->SetLongArrayRegion(env, out, 0, 2, v);
  }
  return out;
}

JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_copyBatch(
    JNIEnv *env, jclass cls, jlong h, jlongArray rowPtr, jintArray cols, jshortArray cnt16, jintArray rowSums32) {
  pin p = pin_get(env, rowPtr), c = pin_get(env, cols), v = pin_get(env, cnt16), r = pin_get(env, rowSums32);
  const int st = cooc_copy_batch(H(h), (int64_t *)p.p, (int32_t *)c.p, NULL, (int16_t *)v.p, NULL, (int32_t *)r.p);
  pin_put(env, r, 1);
  pin_put(env, v, 1);
  pin_put(env, c, 1);
  pin_put(env, p, 1);
  check(env, H(h), st);
}

JNIEXPORT void JNICALL Java_com_github_uce_flinkcooccurrences_CoocNative_topKItems(
    JNIEnv *env, jclass cls, jlong h, jint k, jint flags, jintArray items, jintArray sizes, jintArray values,
    jdoubleArray scores) {
  const jsize n = (*env)->GetArrayLength(env, items);
  pin i = pin_get(env, items), z = pin_get(env, sizes), v = pin_get(env, values), s = pin_get(env, scores);
  const int st = cooc_topk_items(H(h), k, flags, n, (const int32_t *)i.p, (int32_t *)z.p, (int32_t *)v.p,
                                 (double *)s.p);
  pin_put(env, s, 1);
  pin_put(env, v, 1);
  pin_put(env, z, 1);
  pin_put(env, i, 0);
  check(env, H(h), st);
}
