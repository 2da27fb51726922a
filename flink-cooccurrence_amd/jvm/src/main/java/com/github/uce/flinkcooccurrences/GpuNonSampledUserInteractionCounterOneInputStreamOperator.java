package com.github.uce.flinkcooccurrences;

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
 * Drop-in for {@link NonSampledUserInteractionCounterOneInputStreamOperator} (same class shape,
 * constructor arguments, output type and side-output tags, NonSampled...java:31-34,41-46,61,174-176)
 * whose pair expansion and per-window reduction run on an MI355X through libcooc_hip.so.
 *
 * <p>Keyed state moves to the device: the per-user histories of this subtask live in the handle.
 * processElement only buffers the record; processWatermark hands the batch to the device (late
 * records are dropped there, NonSampled...java:89-91) and emits every window the watermark closes,
 * already reduced:
 * <ul>
 *   <li>{@code itemCooccurrences}: one {@link ItemCooccurrences} per (row, column) of the window's delta
 *   rows with {@code increment = (short) count}, so the reference's ItemRowAggregator (addTo,
 *   ItemRowAggregator.java:26-31) rebuilds the same Int2ShortOpenHashMap: addTo is modular, so one
 *   wrapped add of the reduced count equals the reference's count of +1 adds;</li>
 *   <li>{@code rowSums}: one Tuple2(item, delta) per row with a non-zero int delta (RowSumAggregator.java:25-27,66).</li>
 * </ul>
 * Every record carries the window's maxTimestamp (NonSampled...java:115,126-127).  With parallelism p,
 * each subtask owns a user shard (keyBy(0) upstream) and the GPU devices[subtask % devices.length];
 * the downstream keyBy(item) aggregators sum the shards' partial rows exactly as before.
 *
 * <p>Wiring (FlinkCooccurrences.java:70-74):
 * <pre>
 *   interactionStream.keyBy(0).transform("GpuNonSampledUserInteractionCounter",
 *       GpuNonSampledUserInteractionCounterOneInputStreamOperator.getOutputType(),
 *       new GpuNonSampledUserInteractionCounterOneInputStreamOperator(windowSize, windowUnit, nItems, devices));
 * </pre>
 * Uncompiled in the build container (no JDK, Flink 1.3.2 jars absent).
 */
public class GpuNonSampledUserInteractionCounterOneInputStreamOperator
    extends AbstractStreamOperator<Void>
    implements OneInputStreamOperator<Tuple3<Integer, Integer, Long>, Void> {

  private static final long serialVersionUID = 4120558829541227043L;

  @SuppressWarnings("serial")
  private static final OutputTag<ItemCooccurrences> ITEM_TAG =
      new OutputTag<ItemCooccurrences>("itemCooccurrences") {};

  @SuppressWarnings("serial")
  private static final OutputTag<Tuple2<Integer, Integer>> ROW_SUM_TAG =
      new OutputTag<Tuple2<Integer, Integer>>("rowSums") {};

  private final long windowSizeMs;
  private final int nItems;
  private final int[] devices;

  private transient long handle;
  private transient int buffered;
  private transient int[] users;
  private transient int[] items;
  private transient long[] timestamps;
  private transient long[] info;
  private transient Tuple2<Integer, Integer> rowSumsReuse;
  private transient StreamRecord<Tuple2<Integer, Integer>> rowSumsOutputRecord;
  private transient ItemCooccurrences itemCooccurrencesReuse;
  private transient StreamRecord<ItemCooccurrences> itemCooccurrencesOutputRecord;
  private transient IntCounter lateElements;
  private transient LongCounter observedCooccurrences;

  GpuNonSampledUserInteractionCounterOneInputStreamOperator(int windowSize, TimeUnit windowUnit, int nItems,
      int[] devices) {
    this.windowSizeMs = windowUnit.toMillis(windowSize);
    this.nItems = nItems;
    this.devices = devices.clone();
  }

  @Override
  public void open() throws Exception {
    super.open();
    this.handle = CoocNative.create(devices, getRuntimeContext().getIndexOfThisSubtask(), nItems, 0, 0,
        windowSizeMs, (short) 0);
    this.users = new int[1 << 16];
    this.items = new int[1 << 16];
    this.timestamps = new long[1 << 16];
    this.info = new long[6];
    this.rowSumsReuse = new Tuple2<>();
    this.rowSumsOutputRecord = new StreamRecord<>(rowSumsReuse);
    this.itemCooccurrencesReuse = new ItemCooccurrences();
    this.itemCooccurrencesOutputRecord = new StreamRecord<>(itemCooccurrencesReuse);
    this.lateElements = getRuntimeContext().getIntCounter("UserInteractionCounterLateElements");
    this.observedCooccurrences = getRuntimeContext().getLongCounter("UserInteractionCounterObservedCooccurrences");
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

  /** The fired window's delta rows and row sums, on the reference's two side outputs. */
  private void emitWindow() {
    final long timestamp = info[0];
    final int nnz = (int) info[1];
    final int nRows = (int) info[3];
    rowSumsOutputRecord.setTimestamp(timestamp);
    itemCooccurrencesOutputRecord.setTimestamp(timestamp);

    final int[] rows = new int[nRows];
    final long[] rowPtr = new long[nRows + 1];
    final int[] cols = new int[nnz];
    final short[] cnt16 = new short[nnz];
    CoocNative.copyDelta(handle, rows, rowPtr, cols, cnt16);
    for (int r = 0; r < nRows; r++) {
      for (int j = (int) rowPtr[r]; j < (int) rowPtr[r + 1]; j++) {
        itemCooccurrencesReuse.setFields(rows[r], cols[j], cnt16[j]);
        output.collect(ITEM_TAG, itemCooccurrencesOutputRecord);
      }
    }

    final int[] sumItems = new int[nRows];
    final int[] delta32 = new int[nRows];
    CoocNative.copyRowSums(handle, sumItems, delta32);
    for (int r = 0; r < nRows; r++) {
      if (delta32[r] != 0) {
        rowSumsReuse.setFields(sumItems[r], delta32[r]);
        output.collect(ROW_SUM_TAG, rowSumsOutputRecord);
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

  // -------------------------------------------------------------------------------------------------------------------

  static TypeInformation<Void> getOutputType() {
    return new TypeHint<Void>() {}.getTypeInfo();
  }
}
