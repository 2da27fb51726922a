package com.github.uce.flinkcooccurrences;

import it.unimi.dsi.fastutil.ints.Int2ShortOpenHashMap;
import java.util.concurrent.TimeUnit;
import org.apache.flink.api.common.accumulators.IntCounter;
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
 * ({@link GpuCooccurrenceJob#topKOwned}); {@link GpuOwnedCooccurrenceTopKOperator} rescores on the device too.
 *
 * <p>The communicator rendezvous (an id per execution attempt, created by subtask 0 in open()) and the window
 * every subtask fires together are {@link OwnedExchange}'s.  The owned rows stream out in row ranges
 * ({@link CoocBatchReader}: an owner's ~4e9 entries at C3 never need one Java array).  Uncompiled here (no
 * JDK); tests/test_owned_operator_replay.py replays its C-ABI call sequence on two subtasks against the oracle.
 */
public class GpuOwnedCooccurrenceRowsOperator
    extends AbstractStreamOperator<Void>
    implements OneInputStreamOperator<Tuple3<Integer, Integer, Long>, Void> {

  private static final long serialVersionUID = 2281937356412208855L;

  private final long windowSizeMs;
  private final int nItems;
  private final int[] devices;
  private final String rendezvousDir;

  private transient long handle;
  private transient OwnedExchange exchange;
  private transient CoocBatchReader reader;
  private transient IntCounter lateElements;
  private transient LongCounter observedCooccurrences;
  private transient LongCounter rowSumCounter;

  GpuOwnedCooccurrenceRowsOperator(int windowSize, TimeUnit windowUnit, int nItems, int[] devices,
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
    final byte[] commId = OwnedExchange.rendezvous(rendezvousDir,
        getContainingTask().getEnvironment().getJobID().toString(), getRuntimeContext().getAttemptNumber(), subtask);
    this.handle = CoocNative.create(devices, subtask, nItems, 0, 0, windowSizeMs, (short) 0);
    CoocNative.commInit(handle, commId, subtask, world);
    this.exchange = new OwnedExchange(handle, windowSizeMs, world);
    this.reader = new CoocBatchReader();
    this.lateElements = getRuntimeContext().getIntCounter("UserInteractionCounterLateElements");
    this.observedCooccurrences = getRuntimeContext().getLongCounter("UserInteractionCounterObservedCooccurrences");
    this.rowSumCounter = getRuntimeContext().getLongCounter("RowSumProcessWindowRowSum");
  }

  @Override
  public void processElement(StreamRecord<Tuple3<Integer, Integer, Long>> element) throws Exception {
    if (!exchange.add(element.getValue().f0, element.getValue().f1, element.getTimestamp())) {
      lateElements.add(1);  // NonSampled...java:89-91
    }
  }

  @Override
  public void processWatermark(Watermark mark) throws Exception {
    final long ts = exchange.fireAt(mark.getTimestamp());  // (collective over the subtasks)
    if (ts != Long.MIN_VALUE) {
      emitOwnedRows(ts);
    }
    super.processWatermark(mark);
  }

  /** The exchange, then one Int2ShortOpenHashMap per owned row and its int row sum, ascending items. */
  private void emitOwnedRows(long timestamp) {
    final long[] res = exchange.countOwned();  // {nnz, observed, rows, job observed}
    reader.forEachRow(handle, nItems, (item, cols, cnt16, from, to, rowSum32) -> {
      if (to > from) {  // ItemRowAggregator.java:50-56: one map per item with a row
        final Int2ShortOpenHashMap row = new Int2ShortOpenHashMap(to - from);
        for (int j = from; j < to; j++) {
          row.put(cols[j], cnt16[j]);
        }
        output.collect(GpuNonSampledCooccurrenceRowsOperator.ROWS_TAG, new StreamRecord<>(Tuple2.of(item, row), timestamp));
      }
      if (rowSum32 != 0) {  // RowSumAggregator.java:66 (non-owned rows are 0 here)
        rowSumCounter.add(rowSum32);
        output.collect(GpuNonSampledCooccurrenceRowsOperator.ROW_SUM_TAG,
            new StreamRecord<>(Tuple2.of(item, rowSum32), timestamp));
      }
    });
    observedCooccurrences.add(res[1]);  // this subtask's owned pairs: the p accumulators sum to the job's
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
