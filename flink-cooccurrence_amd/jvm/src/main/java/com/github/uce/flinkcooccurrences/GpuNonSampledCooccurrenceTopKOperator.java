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

/**
 * The whole {@code --skip-cuts} graph between keyBy(user) and the sink on one MI355X: the pair emitter
 * (NonSampledUserInteractionCounterOneInputStreamOperator, FlinkCooccurrences.java:65-74), the two keyed
 * window reducers (ItemRowAggregator / RowSumAggregator, :135-157) AND the rescorer
 * (ItemRowRescorerTwoInputStreamOperator(short topK), :162-167).  Its output is the rescorer's: for every
 * item whose row changed in a window, one {@code Tuple2<Integer, IntDoublePriorityQueue>} with the row's
 * LLR top-k (ItemRowRescorer...java:195-226), timestamped with the window's maxTimestamp.  The device keeps
 * the global rows, row sums and observed total (ItemRowRescorer...java:33-41,144-179) and scores every
 * touched row (LogLikelihood.java:41-57, the :238 k22); each heap leaves as cooc_copy_window_topk's
 * IntDoublePriorityQueue layout (positions 1..size, IntDoublePriorityQueue.java:215-242) and is rebuilt
 * here with add() in that order, which keeps the layout (every parent is already <= its children).
 * Like the reference, one queue and one record are reused for every output (ItemRowRescorer...java:42-68);
 * rows are scored in the device's column order (cooc_copy_column_order), where the reference iterates
 * its hash map's slot order: ties at the k-th score may pick other items, as between two fastutil builds.
 * Without a rendezvousDir one subtask holds every user (the graph sets parallelism 1 on it): the resident
 * global state is the rescorer's, which the reference also keeps whole per item.  With one, p subtasks each
 * hold a keyBy(user) shard and the rows they own (a mod p): the p handles join one communicator and every
 * window's exchange runs in the library (cooc_op_process_watermark is collective: partial delta rows to their
 * owners, row sums and the window's pairs all-reduced -- the broadcast row-sum stream of
 * FlinkCooccurrences.java:163 -- and the window agreed by an all-gather); each subtask rescores and emits its
 * owned touched rows, so every item's queue appears on exactly one subtask.  Uncompiled in the build container
 * (no JDK, Flink 1.3.2 / fastutil jars absent); tests/test_boundary_sequence.py replays its C-ABI call
 * sequence at p = 1, tests/test_streaming_multiproc.py the same sequence on two subtasks.
 */
public class GpuNonSampledCooccurrenceTopKOperator
    extends AbstractStreamOperator<Tuple2<Integer, IntDoublePriorityQueue>>
    implements OneInputStreamOperator<Tuple3<Integer, Integer, Long>, Tuple2<Integer, IntDoublePriorityQueue>> {

  private static final long serialVersionUID = 2897354195320881723L;

  private final long windowSizeMs;
  private final int nItems;
  private final int[] devices;
  private final short topK;
  private final String rendezvousDir;  // null: one subtask

  private transient long handle;
  private transient int buffered;
  private transient int[] users;
  private transient int[] items;
  private transient long[] timestamps;
  private transient long[] info;
  private transient long[] counters;
  private transient IntDoublePriorityQueue topKReuse;
  private transient Tuple2<Integer, IntDoublePriorityQueue> itemTopKReuse;
  private transient StreamRecord<Tuple2<Integer, IntDoublePriorityQueue>> outputRecordReuse;
  private transient IntCounter lateElements;
  private transient LongCounter observedCooccurrences;
  private transient LongCounter rowSumCounter;
  private transient LongCounter rescoredItems;

  GpuNonSampledCooccurrenceTopKOperator(int windowSize, TimeUnit windowUnit, int nItems, int[] devices, short topK) {
    this(windowSize, windowUnit, nItems, devices, topK, null);
  }

  /** rendezvousDir: a directory every subtask of the node reads (the communicator id per attempt). */
  GpuNonSampledCooccurrenceTopKOperator(int windowSize, TimeUnit windowUnit, int nItems, int[] devices, short topK,
      String rendezvousDir) {
    if (topK <= 0) {  // ItemRowRescorerTwoInputStreamOperator.java:52-54
      throw new IllegalArgumentException(topK + " is <= 0");
    }
    this.windowSizeMs = windowUnit.toMillis(windowSize);
    this.nItems = nItems;
    this.devices = devices.clone();
    this.topK = topK;
    this.rendezvousDir = rendezvousDir;
  }

  @Override
  public void open() throws Exception {
    super.open();
    final int subtask = getRuntimeContext().getIndexOfThisSubtask();
    final int world = getRuntimeContext().getNumberOfParallelSubtasks();
    this.handle = CoocNative.create(devices, subtask, nItems, topK, 0, windowSizeMs, (short) 0);
    if (rendezvousDir != null && world > 1) {  // owned rows: the windows' exchange inside the library
      CoocNative.commInit(handle, OwnedExchange.rendezvous(rendezvousDir,
          getContainingTask().getEnvironment().getJobID().toString(), getRuntimeContext().getAttemptNumber(),
          subtask), subtask, world);
    }
    this.users = new int[1 << 16];
    this.items = new int[1 << 16];
    this.timestamps = new long[1 << 16];
    this.info = new long[6];
    this.counters = new long[5];
    this.topKReuse = new IntDoublePriorityQueue(topK);
    this.itemTopKReuse = new Tuple2<>();
    this.outputRecordReuse = new StreamRecord<>(itemTopKReuse);
    this.lateElements = getRuntimeContext().getIntCounter("UserInteractionCounterLateElements");
    this.observedCooccurrences = getRuntimeContext().getLongCounter("UserInteractionCounterObservedCooccurrences");
    this.rowSumCounter = getRuntimeContext().getLongCounter("RowSumProcessWindowRowSum");
    this.rescoredItems = getRuntimeContext().getLongCounter("ItemRowRescorerRescoredItems");
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
    CoocNative.counters(handle, counters);
    final long rowSumsBefore = counters[2], rescoredBefore = counters[3];
    while (CoocNative.processWatermark(handle, mark.getTimestamp(), info)) {
      emitTopK();
    }
    CoocNative.counters(handle, counters);
    rowSumCounter.add(counters[2] - rowSumsBefore);      // RowSumAggregator.java:50,67
    rescoredItems.add(counters[3] - rescoredBefore);      // ItemRowRescorer...java:60,169
    super.processWatermark(mark);
  }

  /** One fired window: every rescored row's heap, ItemRowRescorer...java:224-226. */
  private void emitTopK() {
    final long timestamp = info[0];
    final int k = (int) info[4], nTopK = (int) info[5];
    observedCooccurrences.add(info[2]);
    if (nTopK == 0) {
      return;
    }
    final int[] rows = new int[nTopK];
    final int[] sizes = new int[nTopK];
    final int[] values = new int[nTopK * k];
    final double[] scores = new double[nTopK * k];
    CoocNative.copyTopK(handle, rows, sizes, values, scores);
    outputRecordReuse.setTimestamp(timestamp);
    for (int r = 0; r < nTopK; r++) {
      topKReuse.reset();
      for (int i = 0; i < sizes[r]; i++) {
        topKReuse.add(values[r * k + i], scores[r * k + i]);  // heap order in, the same heap out
      }
      itemTopKReuse.setFields(rows[r], topKReuse);
      output.collect(outputRecordReuse);
    }
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

  static TypeInformation<Tuple2<Integer, IntDoublePriorityQueue>> getOutputType() {
    return new TypeHint<Tuple2<Integer, IntDoublePriorityQueue>>() {}.getTypeInfo();
  }
}
