package com.github.uce.flinkcooccurrences;

import it.unimi.dsi.fastutil.ints.Int2ShortOpenHashMap;
import java.util.Arrays;
import java.util.concurrent.TimeUnit;
import org.apache.flink.api.common.accumulators.IntCounter;
import org.apache.flink.api.common.accumulators.LongCounter;
import org.apache.flink.api.common.typeinfo.TypeHint;
import org.apache.flink.api.common.typeinfo.TypeInformation;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.api.java.tuple.Tuple3;
import org.apache.flink.streaming.api.operators.AbstractStreamOperator;
import org.apache.flink.streaming.api.operators.OneInputStreamOperator;
import org.apache.flink.streaming.api.watermark.Watermark;
import org.apache.flink.streaming.runtime.streamrecord.StreamRecord;
import org.apache.flink.util.OutputTag;

/**
 * The pair emitter AND both keyed window reducers of the {@code --skip-cuts} graph on an MI355X: it
 * replaces NonSampledUserInteractionCounterOneInputStreamOperator (FlinkCooccurrences.java:65-74) plus
 * the ItemRowAggregator and RowSumAggregator windows (FlinkCooccurrences.java:135-157).  No
 * ItemCooccurrences record is created: every window the watermark closes leaves the device already
 * reduced, on two side outputs whose records are exactly what the two reference windows emit:
 * <ul>
 *   <li>{@link #ROWS_TAG}: one {@code Tuple2<Integer, Int2ShortOpenHashMap>} per item with a delta row
 *   (ItemCooccurrenceRowWindowFunction.process, ItemRowAggregator.java:50-56): the map holds every
 *   touched column with the count as a Java short (addTo wraps, ItemRowAggregator.java:29);</li>
 *   <li>{@link #ROW_SUM_TAG}: one {@code Tuple2<Integer, Integer>} per item whose int row-sum delta is
 *   non-zero (RowSumProcessWindow.process, RowSumAggregator.java:54-71), and the
 *   RowSumProcessWindowRowSum accumulator (:50,67).</li>
 * </ul>
 * Every record carries the window's maxTimestamp, as a window operator's output does.  With one subtask
 * the rows and row sums are final and feed ItemRowRescorerTwoInputStreamOperator directly.  With p > 1
 * each subtask holds a user shard (keyBy(0)); then either
 * <ul>
 *   <li>a rendezvousDir is given: the p handles join one communicator (the attempt's id from subtask 0,
 *   {@link OwnedExchange#rendezvous}) and every window's exchange runs inside the library
 *   (cooc_op_process_watermark is collective: partial delta rows to their owners a mod p over RCCL, row
 *   sums all-reduced, the window agreed by an all-gather); each subtask emits the complete rows it owns and
 *   the job's row sums of those rows, which feed the rescorer with no merge windows; or</li>
 *   <li>its rows are partial and one keyed reduce per stream ({@link GpuCooccurrenceJob}) sums the p
 *   partial rows per item and window -- p records per row instead of one record per ordered pair.</li>
 * </ul>  Emitted objects are fresh (the rescorer buffers them by
 * timestamp, ItemRowRescorer...java:83-113, and object reuse is on, FlinkCooccurrences.java:44).
 * Uncompiled in the build container (no JDK, Flink 1.3.2 / fastutil jars absent); the C-ABI call
 * sequence it makes is replayed by tests/test_boundary_sequence.py.
 */
public class GpuNonSampledCooccurrenceRowsOperator
    extends AbstractStreamOperator<Void>
    implements OneInputStreamOperator<Tuple3<Integer, Integer, Long>, Void> {

  private static final long serialVersionUID = 7321170436981573315L;

  @SuppressWarnings("serial")
  static final OutputTag<Tuple2<Integer, Int2ShortOpenHashMap>> ROWS_TAG =
      new OutputTag<Tuple2<Integer, Int2ShortOpenHashMap>>("itemCooccurrenceRows") {};

  @SuppressWarnings("serial")
  static final OutputTag<Tuple2<Integer, Integer>> ROW_SUM_TAG =
      new OutputTag<Tuple2<Integer, Integer>>("rowSumsReduced") {};

  private final long windowSizeMs;
  private final int nItems;
  private final int[] devices;
  private final String rendezvousDir;  // null: partial rows at p > 1 (merged downstream)

  private transient long handle;
  private transient int buffered;
  private transient int[] users;
  private transient int[] items;
  private transient long[] timestamps;
  private transient long[] info;
  private transient CoocWindowReader reader;
  private transient IntCounter lateElements;
  private transient LongCounter observedCooccurrences;
  private transient LongCounter rowSumCounter;

  GpuNonSampledCooccurrenceRowsOperator(int windowSize, TimeUnit windowUnit, int nItems, int[] devices) {
    this(windowSize, windowUnit, nItems, devices, null);
  }

  /** rendezvousDir: a directory every subtask of the node reads (the communicator id per attempt). */
  GpuNonSampledCooccurrenceRowsOperator(int windowSize, TimeUnit windowUnit, int nItems, int[] devices,
      String rendezvousDir) {
    this.windowSizeMs = windowUnit.toMillis(windowSize);
    this.nItems = nItems;
    this.devices = devices.clone();
    this.rendezvousDir = rendezvousDir;
  }

  @Override
  public void open() throws Exception {
    super.open();
    final int subtask = getRuntimeContext().getIndexOfThisSubtask();
    final int world = getRuntimeContext().getNumberOfParallelSubtasks();
    this.handle = CoocNative.create(devices, subtask, nItems, 0, 0, windowSizeMs, (short) 0);
    if (rendezvousDir != null && world > 1) {  // owned rows: the windows' exchange inside the library
      CoocNative.commInit(handle, OwnedExchange.rendezvous(rendezvousDir,
          getContainingTask().getEnvironment().getJobID().toString(), getRuntimeContext().getAttemptNumber(),
          subtask), subtask, world);
    }
    this.users = new int[1 << 16];
    this.items = new int[1 << 16];
    this.timestamps = new long[1 << 16];
    this.info = new long[6];
    this.reader = new CoocWindowReader();
    this.lateElements = getRuntimeContext().getIntCounter("UserInteractionCounterLateElements");
    this.observedCooccurrences = getRuntimeContext().getLongCounter("UserInteractionCounterObservedCooccurrences");
    this.rowSumCounter = getRuntimeContext().getLongCounter("RowSumProcessWindowRowSum");
  }

  @Override
  public void processElement(StreamRecord<Tuple3<Integer, Integer, Long>> element) throws Exception {
    if (buffered == users.length) {
      users = Arrays.copyOf(users, 2 * buffered);
      items = Arrays.copyOf(items, 2 * buffered);
      timestamps = Arrays.copyOf(timestamps, 2 * buffered);
    }
    final Tuple3<Integer, Integer, Long> interaction = element.getValue();
    users[buffered] = interaction.f0;
    items[buffered] = interaction.f1;
    timestamps[buffered] = element.getTimestamp();
    buffered++;
  }

  @Override
  public void processWatermark(Watermark mark) throws Exception {
    if (buffered > 0) {
      lateElements.add((int) CoocNative.processElements(handle, buffered, users, items, timestamps));
      buffered = 0;
    }
    while (CoocNative.processWatermark(handle, mark.getTimestamp(), info)) {
      emitWindow();
    }
    super.processWatermark(mark);
  }

  private void emitWindow() {
    final long timestamp = info[0];
    final int nRows = (int) info[3];
    reader.forEachRow(handle, nRows, (item, cols, cnt16, from, to) -> {
      final Int2ShortOpenHashMap row = new Int2ShortOpenHashMap(to - from);
      for (int j = from; j < to; j++) {
        row.put(cols[j], cnt16[j]);
      }
      output.collect(ROWS_TAG, new StreamRecord<>(Tuple2.of(item, row), timestamp));
    });
    final int[] sumItems = new int[nRows];
    final int[] delta32 = new int[nRows];
    CoocNative.copyRowSums(handle, sumItems, delta32);
    for (int r = 0; r < nRows; r++) {
      if (delta32[r] != 0) {  // RowSumAggregator.java:66
        rowSumCounter.add(delta32[r]);
        output.collect(ROW_SUM_TAG, new StreamRecord<>(Tuple2.of(sumItems[r], delta32[r]), timestamp));
      }
    }
    observedCooccurrences.add(info[2]);
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

  static TypeInformation<Void> getOutputType() {
    return new TypeHint<Void>() {}.getTypeInfo();
  }
}
