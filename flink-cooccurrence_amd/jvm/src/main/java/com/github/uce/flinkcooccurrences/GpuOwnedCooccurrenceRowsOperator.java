package com.github.uce.flinkcooccurrences;

import it.unimi.dsi.fastutil.ints.Int2ShortOpenHashMap;
import java.util.Arrays;
import java.util.concurrent.TimeUnit;
import org.apache.flink.api.common.accumulators.LongCounter;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.api.java.tuple.Tuple3;
import org.apache.flink.streaming.api.operators.AbstractStreamOperator;
import org.apache.flink.streaming.api.operators.OneInputStreamOperator;
import org.apache.flink.streaming.api.watermark.Watermark;
import org.apache.flink.streaming.runtime.streamrecord.StreamRecord;

/**
 * The rows operator for p > 1 subtasks of a ONE-window job (the C3 / C5 configs: a bounded log whose
 * timestamps fall in one tumbling window), with the reference's keyBy(item) shuffle
 * (FlinkCooccurrences.java:138-157: p partial rows per item summed by ItemRowAggregator / RowSumAggregator
 * windows) replaced by the library's exchange over RCCL (cooc_count_owned_host): every subtask holds a user
 * shard (keyBy(0)); when the watermark closes the window, the subtasks' handles all-reduce the item
 * frequencies, agree on the row-owner map, exchange the histories over xGMI and each counts the rows it
 * owns over every user.  Rows are complete on their owner, so the side outputs ({@link
 * GpuNonSampledCooccurrenceRowsOperator#ROWS_TAG}, {@link GpuNonSampledCooccurrenceRowsOperator#ROW_SUM_TAG})
 * carry final rows and row sums and feed ItemRowRescorerTwoInputStreamOperator with no merge
 * ({@link GpuCooccurrenceJob#topKOwned}).
 *
 * <p>The communicator id is created once in the job's main() ({@link CoocNative#commUniqueId}) and handed to
 * every subtask in the constructor; open() joins it as subtask i of p.  A record whose timestamp falls in
 * another window fails the job (IllegalStateException): multi-window streams keep the partial-row path.
 * The owned rows are copied in one call, so a subtask's owned entries must fit a Java array (2^31 - 1);
 * larger results are read through the Panama path (INTEGRATION.md §4).  Uncompiled here (no JDK); the
 * C-ABI sequence it makes is tests/test_multiproc_gpu.py's "library_host" case.
 */
public class GpuOwnedCooccurrenceRowsOperator
    extends AbstractStreamOperator<Void>
    implements OneInputStreamOperator<Tuple3<Integer, Integer, Long>, Void> {

  private static final long serialVersionUID = 2281937356412208855L;

  private final long windowSizeMs;
  private final int nItems;
  private final int[] devices;
  private final byte[] commId;

  private transient long handle;
  private transient int buffered;
  private transient int[] users;
  private transient int[] items;
  private transient long windowStart;
  private transient boolean fired;
  private transient LongCounter observedCooccurrences;
  private transient LongCounter rowSumCounter;

  GpuOwnedCooccurrenceRowsOperator(int windowSize, TimeUnit windowUnit, int nItems, int[] devices, byte[] commId) {
    this.windowSizeMs = windowUnit.toMillis(windowSize);
    this.nItems = nItems;
    this.devices = devices.clone();
    this.commId = commId.clone();
  }

  @Override
  public void open() throws Exception {
    super.open();
    final int subtask = getRuntimeContext().getIndexOfThisSubtask();
    this.handle = CoocNative.create(devices, subtask, nItems, 0, 0, windowSizeMs, (short) 0);
    CoocNative.commInit(handle, commId, subtask, getRuntimeContext().getNumberOfParallelSubtasks());
    this.users = new int[1 << 16];
    this.items = new int[1 << 16];
    this.windowStart = Long.MIN_VALUE;
    this.observedCooccurrences = getRuntimeContext().getLongCounter("UserInteractionCounterObservedCooccurrences");
    this.rowSumCounter = getRuntimeContext().getLongCounter("RowSumProcessWindowRowSum");
  }

  @Override
  public void processElement(StreamRecord<Tuple3<Integer, Integer, Long>> element) throws Exception {
    // TumblingEventTimeWindows' start (offset 0): the one window this operator serves
    final long ts = element.getTimestamp();
    final long start = ts - Math.floorMod(ts, windowSizeMs);
    if (windowStart == Long.MIN_VALUE) {
      windowStart = start;
    } else if (start != windowStart || fired) {
      throw new IllegalStateException("GpuOwnedCooccurrenceRowsOperator serves one window; record at " + ts);
    }
    if (buffered == users.length) {
      users = Arrays.copyOf(users, 2 * buffered);
      items = Arrays.copyOf(items, 2 * buffered);
    }
    users[buffered] = element.getValue().f0;
    items[buffered] = element.getValue().f1;
    buffered++;
  }

  @Override
  public void processWatermark(Watermark mark) throws Exception {
    // every subtask reaches the window's end (the final watermark of a bounded source at the latest) and
    // takes part in the exchange, also one that holds no users
    final long maxTimestamp = windowStart == Long.MIN_VALUE ? Long.MAX_VALUE - 1 : windowStart + windowSizeMs - 1;
    if (!fired && mark.getTimestamp() >= maxTimestamp) {
      fired = true;
      emitOwnedRows(maxTimestamp);
    }
    super.processWatermark(mark);
  }

  /** CSR of the shard's users (a user's items in arrival order), the exchange, the owned rows out. */
  private void emitOwnedRows(long timestamp) {
    final int[] order = new int[buffered];
    final int[] userIds = Arrays.copyOf(users, buffered);
    final Integer[] idx = new Integer[buffered];
    for (int i = 0; i < buffered; i++) {
      idx[i] = i;
    }
    Arrays.sort(idx, (x, y) -> userIds[x] != userIds[y] ? Integer.compare(userIds[x], userIds[y]) : Integer.compare(x, y));
    int nUsers = 0;
    for (int i = 0; i < buffered; i++) {
      order[i] = items[idx[i]];
      if (i == 0 || userIds[idx[i]] != userIds[idx[i - 1]]) {
        nUsers++;
      }
    }
    final long[] userPtr = new long[nUsers + 1];
    for (int i = 0, u = 0; i < buffered; i++) {
      if (i > 0 && userIds[idx[i]] != userIds[idx[i - 1]]) {
        userPtr[++u] = i;
      }
    }
    userPtr[nUsers] = buffered;
    final long[] res = CoocNative.countOwned(handle, userPtr, order);  // {nnz, observed, rows, job observed}
    final long[] rowPtr = new long[nItems + 1];
    final int[] cols = new int[Math.toIntExact(res[0])];
    final short[] cnt16 = new short[cols.length];
    final int[] rowSums32 = new int[nItems];
    CoocNative.copyBatch(handle, rowPtr, cols, cnt16, rowSums32);
    for (int a = 0; a < nItems; a++) {
      final int from = (int) rowPtr[a], to = (int) rowPtr[a + 1];
      if (to > from) {  // ItemRowAggregator.java:50-56: one map per item with a row
        final Int2ShortOpenHashMap row = new Int2ShortOpenHashMap(to - from);
        for (int j = from; j < to; j++) {
          row.put(cols[j], cnt16[j]);
        }
        output.collect(GpuNonSampledCooccurrenceRowsOperator.ROWS_TAG, new StreamRecord<>(Tuple2.of(a, row), timestamp));
      }
      if (rowSums32[a] != 0) {  // RowSumAggregator.java:66 (non-owned rows are 0 here)
        rowSumCounter.add(rowSums32[a]);
        output.collect(GpuNonSampledCooccurrenceRowsOperator.ROW_SUM_TAG,
            new StreamRecord<>(Tuple2.of(a, rowSums32[a]), timestamp));
      }
    }
    observedCooccurrences.add(res[1]);  // this subtask's owned pairs: the p accumulators sum to the job's
    buffered = 0;
  }

  @Override
  public void close() throws Exception {
    try {
      if (handle != 0) {
        CoocNative.destroy(handle);
        handle = 0;
      }
    } finally {
      super.close();
    }
  }
}
