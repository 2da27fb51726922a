package com.github.uce.flinkcooccurrences;

/**
 * Streams the delta rows of the window a handle just fired (CoocNative.processWatermark) out of the
 * device in row ranges: CoocNative.copyDeltaRows once, then CoocNative.copyDeltaRange for runs of rows
 * whose entries fit {@link #MAX_RANGE_ENTRIES}.  A C3-sized window holds ~7e9 entries per GPU, more
 * than one Java array can (2^31 - 1); a single row never holds more than nItems.
 */
final class CoocWindowReader {

  /** Entries per range copy (64 MiB of cols + 32 MiB of counts). */
  static final int MAX_RANGE_ENTRIES = 1 << 24;

  /** One delta row: entries [from, to) of cols / cnt16 (valid only during the call). */
  interface RowConsumer {
    void row(int item, int[] cols, short[] cnt16, int from, int to);
  }

  private int[] cols = new int[1 << 16];
  private short[] cnt16 = new short[1 << 16];

  /** Calls consumer for every delta row of the fired window, in ascending item order. */
  void forEachRow(long handle, int nRows, RowConsumer consumer) {
    final int[] rows = new int[nRows];
    final long[] rowPtr = new long[nRows + 1];
    CoocNative.copyDeltaRows(handle, rows, rowPtr);
    int r0 = 0;
    while (r0 < nRows) {
      int r1 = r0 + 1;
      while (r1 < nRows && rowPtr[r1 + 1] - rowPtr[r0] <= MAX_RANGE_ENTRIES) {
        r1++;
      }
      final int n = (int) (rowPtr[r1] - rowPtr[r0]);
      if (cols.length < n) {
        cols = new int[n];
        cnt16 = new short[n];
      }
      CoocNative.copyDeltaRange(handle, r0, r1, n, cols, cnt16);
      for (int r = r0; r < r1; r++) {
        consumer.row(rows[r], cols, cnt16, (int) (rowPtr[r] - rowPtr[r0]), (int) (rowPtr[r + 1] - rowPtr[r0]));
      }
      r0 = r1;
    }
  }
}
