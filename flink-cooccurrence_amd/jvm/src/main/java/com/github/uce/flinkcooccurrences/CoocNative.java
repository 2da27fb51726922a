package com.github.uce.flinkcooccurrences;

/**
 * JNI mirror of include/cooc.h (libcooc_jni.so, built from ../../../../../../jni/cooc_jni.c, links
 * libcooc_hip.so).  One handle per Flink subtask; a handle is not thread-safe, handles are
 * independent.  Every native throws IllegalArgumentException for COOC_ERR_ARG and
 * IllegalStateException for any other non-zero status, with cooc_last_error() as the message --
 * the reference's error behaviour (e.g. ItemRowRescorerTwoInputStreamOperator.java:52-54,72-79).
 *
 * Uncompiled in the build container (no JDK); every entry point it binds is exercised through the
 * same C-ABI by the Python ctypes tests (tests/test_gpu_parity.py, flink-cooccurrence_amd/_lib.py).
 */
final class CoocNative {

  static {
    System.loadLibrary("cooc_jni");
  }

  static final int FLAG_EXACT_SCORES = 1;  // COOC_FLAG_EXACT_SCORES

  private CoocNative() {
  }

  /** cooc_create_on: the handle of subtask {@code subtask} binds to devices[subtask % devices.length]. */
  static native long create(int[] devices, int subtask, int nItems, int topK, int flags, long windowSizeMs,
      short userCut);

  /** cooc_destroy. */
  static native void destroy(long handle);

  /**
   * cooc_op_process_elements: one buffered batch of Tuple3(user, item, timestamp) as parallel arrays
   * (the first n entries).  Late records (timestamp <= the current watermark, NonSampled...java:89-91)
   * are dropped; returns how many.
   */
  static native long processElements(long handle, int n, int[] users, int[] items, long[] timestamps);

  /**
   * cooc_op_process_watermark: fires the next window whose maxTimestamp <= watermark, if any.  On
   * true, info = {ts, nnz, observed, nRows, topK, nTopK} (cooc_window_info) sizes the copy calls.
   */
  static native boolean processWatermark(long handle, long watermark, long[] info);

  /**
   * cooc_copy_window_delta of the fired window, rows only: rows int[nRows] (ascending items with a delta
   * row), rowPtr long[nRows + 1] (their entry offsets).  The entries stream out with copyDeltaRange, so
   * that a window larger than one Java array (2^31 - 1 entries) never needs one.
   */
  static native void copyDeltaRows(long handle, int[] rows, long[] rowPtr);

  /**
   * cooc_copy_window_delta_range: the entries of delta rows [rowBegin, rowEnd) -- cols int[n], cnt16
   * short[n] with n = rowPtr[rowEnd] - rowPtr[rowBegin] -- the window's reduced ItemRowAggregator rows
   * (Int2ShortOpenHashMap values, ItemRowAggregator.java:26-31).
   */
  static native void copyDeltaRange(long handle, int rowBegin, int rowEnd, int n, int[] cols, short[] cnt16);

  /** cooc_copy_window_rowsums: items int[nRows], delta32 int[nRows] (RowSumAggregator values). */
  static native void copyRowSums(long handle, int[] items, int[] delta32);

  /** cooc_copy_window_topk: rows int[nTopK], sizes int[nTopK], values int[nTopK * topK], scores double[...]. */
  static native void copyTopK(long handle, int[] rows, int[] sizes, int[] values, double[] scores);

  /**
   * cooc_op_counters: {UserInteractionCounterLateElements, UserInteractionCounterObservedCooccurrences,
   * RowSumProcessWindowRowSum, ItemRowRescorerRescoredItems, rescorer observed}.
   */
  static native void counters(long handle, long[] out5);

  /**
   * cooc_count_host: one stateless window over CSR histories (userPtr long[nUsers + 1] into items).
   * Returns {nnz, observed}; the result stays on the handle for copyBatch / topKItems.
   */
  static native long[] countBatch(long handle, long[] userPtr, int[] items);

  /** cooc_copy_batch: rowPtr long[nItems + 1], cols int[nnz], cnt16 short[nnz], rowSums32 int[nItems]. */
  static native void copyBatch(long handle, long[] rowPtr, int[] cols, short[] cnt16, int[] rowSums32);

  /**
   * cooc_comm_unique_id: the 128-byte RCCL id of a new communicator (host only: created once in the job's
   * main() and handed to every subtask in its operator's constructor).
   */
  static native byte[] commUniqueId();

  /** cooc_comm_init: the handle joins the communicator as subtask {@code rank} of {@code world} (open()). */
  static native void commInit(long handle, byte[] id, int rank, int world);

  /**
   * cooc_count_owned_host: this subtask's users (userPtr long[nUsers + 1] into items) -> the rows it owns
   * over every subtask's users (item counts all-reduced, owner map, histories exchanged over RCCL, owned
   * rows counted).  Returns {nnz, observed, rows with entries} of the owned rows and the job's observed;
   * the owned rows are then the handle's batch (copyBatch: every other row empty).
   */
  static native long[] countOwned(long handle, long[] userPtr, int[] items);

  /**
   * cooc_copy_batch_range: the entries of batch rows [rowBegin, rowEnd) -- cols int[n], cnt16 short[n] with n =
   * rowPtr[rowEnd] - rowPtr[rowBegin] from copyBatch(rowPtr, null, null, rowSums32) -- ascending columns per row.
   */
  static native void copyBatchRange(long handle, int rowBegin, int rowEnd, int n, int[] cols, short[] cnt16);

  /**
   * cooc_topk_owned_host: after countOwned, the owned rows' row sums all-reduced (the broadcast row-sum stream,
   * FlinkCooccurrences.java:163) and every owned row's LLR top-k on the device; read with copyTopKRange.
   */
  static native void topKOwned(long handle, int k, int flags);

  /** cooc_copy_topk_batch_range: rows [rowBegin, rowEnd): sizes int[n], values int[n * k], scores double[n * k]. */
  static native void copyTopKRange(long handle, int rowBegin, int rowEnd, int k, int[] sizes, int[] values,
      double[] scores);

  /** cooc_comm_allgather_i64: every subtask's value (collective over the handle's communicator), rank order. */
  static native long[] commAllGather(long handle, long value, int world);

  /** cooc_topk_items: topk(handle, items[], k) of the last batch; sizes int[n], values/scores [n * k]. */
  static native void topKItems(long handle, int k, int flags, int[] items, int[] sizes, int[] values,
      double[] scores);
}
