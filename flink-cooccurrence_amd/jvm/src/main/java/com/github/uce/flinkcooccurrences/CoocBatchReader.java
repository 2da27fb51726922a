package com.github.uce.flinkcooccurrences;

/**
 * Streams a handle's batch result (an owner's rows after CoocNative.countOwned) out of the device in row
 * ranges, as CoocWindowReader does for a fired window: CoocNative.copyBatch for the row offsets and int row
 * sums once, then CoocNative.copyBatchRange for runs of rows whose entries fit {@link #maxRangeEntries}.  An
 * owner holds ~4e9 entries at C3 (8 GPUs), more than one Java array can (2^31 - 1); a single row never holds
 * more than nItems.  The heaps of CoocNative.topKOwned stream the same way (forEachTopK).
 */
final class CoocBatchReader {

  /** Entries per range copy by default (64 MiB of cols + 32 MiB of counts). */
  static final int MAX_RANGE_ENTRIES = 1 << 24;
  /** Rows per heap range copy. */
  static final int TOPK_ROWS_PER_RANGE = 1 << 14;

  interface RowConsumer {
    /** One row with entries [from, to) of cols / cnt16 and its int row sum (valid only during the call). */
    void row(int item, int[] cols, short[] cnt16, int from, int to, int rowSum32);
  }

  interface TopKConsumer {
    /** One row's heap: values / scores [from, from + size) in IntDoublePriorityQueue order. */
    void heap(int item, int size, int[] values, double[] scores, int from);
  }

  private final int maxRangeEntries;
  private int[] cols = new int[1 << 16];
  private short[] cnt16 = new short[1 << 16];

  CoocBatchReader() {
    this(MAX_RANGE_ENTRIES);
  }

  CoocBatchReader(int maxRangeEntries) {
    this.maxRangeEntries = maxRangeEntries;
  }

  /** Every row with entries or a non-zero int row sum, ascending item order. */
  void forEachRow(long handle, int nItems, RowConsumer consumer) {
    final long[] rowPtr = new long[nItems + 1];
    final int[] rowSums32 = new int[nItems];
    CoocNative.copyBatch(handle, rowPtr, null, null, rowSums32);
    int r0 = 0;
    while (r0 < nItems) {
      int r1 = r0 + 1;
      while (r1 < nItems && rowPtr[r1 + 1] - rowPtr[r0] <= maxRangeEntries) {
        r1++;
      }
      final int n = (int) (rowPtr[r1] - rowPtr[r0]);
      if (cols.length < n) {
        cols = new int[n];
        cnt16 = new short[n];
      }
      if (n > 0) {
        CoocNative.copyBatchRange(handle, r0, r1, n, cols, cnt16);
      }
      for (int r = r0; r < r1; r++) {
        final int from = (int) (rowPtr[r] - rowPtr[r0]), to = (int) (rowPtr[r + 1] - rowPtr[r0]);
        if (to > from || rowSums32[r] != 0) {
          consumer.row(r, cols, cnt16, from, to, rowSums32[r]);
        }
      }
      r0 = r1;
    }
  }

  /** Every row with a non-empty heap (after CoocNative.topKOwned), ascending item order. */
  static void forEachTopK(long handle, int nItems, int k, TopKConsumer consumer) {
    final int[] sizes = new int[TOPK_ROWS_PER_RANGE];
    final int[] values = new int[TOPK_ROWS_PER_RANGE * k];
    final double[] scores = new double[TOPK_ROWS_PER_RANGE * k];
    for (int r0 = 0; r0 < nItems; r0 += TOPK_ROWS_PER_RANGE) {
      final int r1 = Math.min(nItems, r0 + TOPK_ROWS_PER_RANGE);
      CoocNative.copyTopKRange(handle, r0, r1, k, sizes, values, scores);
      for (int r = r0; r < r1; r++) {
        final int size = sizes[r - r0];
        if (size > 0) {
          consumer.heap(r, size, values, scores, (r - r0) * k);
        }
      }
    }
  }
}
