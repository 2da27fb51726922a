package com.github.uce.flinkcooccurrences;

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
 * C5 on p GPUs through the drop-in: the whole {@code --skip-cuts} graph of a ONE-window job -- the pair emitter
 * (FlinkCooccurrences.java:65-74), the keyBy(item) row / row-sum windows (:135-157) AND the rescorer
 * (ItemRowRescorerTwoInputStreamOperator(short topK), :162-167) -- as p subtasks whose handles exchange over
 * RCCL.  Each subtask holds a keyBy(user) shard; when the window closes ({@link OwnedExchange#fireAt}, the same
 * window on every subtask) its handle counts the rows it owns over every user (cooc_count_owned_host), the
 * owned row sums are all-reduced -- the broadcast row-sum stream of :163 -- and every owned row is rescored on
 * the device against them and the job's observed total (cooc_topk_owned_host: ItemRowRescorer...java:195-241,
 * LogLikelihood.java:41-57 with the :238 k22).  The output is the rescorer's: one {@code Tuple2<Integer,
 * IntDoublePriorityQueue>} per owned row with entries (ItemRowRescorer...java:224-226), timestamped with the
 * window's maxTimestamp; across the p subtasks every row of the window appears exactly once.  Heaps leave the
 * device in row ranges (CoocBatchReader.forEachTopK) in IntDoublePriorityQueue's layout and are rebuilt with
 * add() in that order, which keeps the layout.  Like the reference, one queue and one record are reused.
 * Rows are scored in the device's column order where the reference iterates its hash map's slot order: ties
 * at the k-th score may pick other items, as between two fastutil builds.
 *
 * <p>No partial row or heap crosses the JVM: the job's only host traffic is the records in and the heaps
 * out.  Uncompiled here (no JDK); tests/test_owned_operator_replay.py replays its C-ABI call sequence on two
 * subtasks against the oracle's rescorer.
 */
public class GpuOwnedCooccurrenceTopKOperator
    extends AbstractStreamOperator<Tuple2<Integer, IntDoublePriorityQueue>>
    implements OneInputStreamOperator<Tuple3<Integer, Integer, Long>, Tuple2<Integer, IntDoublePriorityQueue>> {

  private static final long serialVersionUID = 6154098321567734519L;

  private final long windowSizeMs;
  private final int nItems;
  private final int[] devices;
  private final short topK;
  private final String rendezvousDir;

  private transient long handle;
  private transient OwnedExchange exchange;
  private transient IntDoublePriorityQueue topKReuse;
  private transient Tuple2<Integer, IntDoublePriorityQueue> itemTopKReuse;
  private transient StreamRecord<Tuple2<Integer, IntDoublePriorityQueue>> outputRecordReuse;
  private transient IntCounter lateElements;
  private transient LongCounter observedCooccurrences;
  private transient LongCounter rescoredItems;

  GpuOwnedCooccurrenceTopKOperator(int windowSize, TimeUnit windowUnit, int nItems, int[] devices, short topK,
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
    final byte[] commId = OwnedExchange.rendezvous(rendezvousDir,
        getContainingTask().getEnvironment().getJobID().toString(), getRuntimeContext().getAttemptNumber(), subtask);
    this.handle = CoocNative.create(devices, subtask, nItems, topK, 0, windowSizeMs, (short) 0);
    CoocNative.commInit(handle, commId, subtask, world);
    this.exchange = new OwnedExchange(handle, windowSizeMs, world);
    this.topKReuse = new IntDoublePriorityQueue(topK);
    this.itemTopKReuse = new Tuple2<>();
    this.outputRecordReuse = new StreamRecord<>(itemTopKReuse);
    this.lateElements = getRuntimeContext().getIntCounter("UserInteractionCounterLateElements");
    this.observedCooccurrences = getRuntimeContext().getLongCounter("UserInteractionCounterObservedCooccurrences");
    this.rescoredItems = getRuntimeContext().getLongCounter("ItemRowRescorerRescoredItems");
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
      final long[] res = exchange.countOwned();  // {nnz, observed, rows, job observed}
      observedCooccurrences.add(res[1]);
      CoocNative.topKOwned(handle, topK, 0);
      outputRecordReuse.setTimestamp(ts);
      CoocBatchReader.forEachTopK(handle, nItems, topK, (item, size, values, scores, from) -> {
        topKReuse.reset();
        for (int i = 0; i < size; i++) {
          topKReuse.add(values[from + i], scores[from + i]);  // heap order in, the same heap out
        }
        itemTopKReuse.setFields(item, topKReuse);
        output.collect(outputRecordReuse);
        rescoredItems.add(1L);  // ItemRowRescorer...java:60,169
      });
    }
    super.processWatermark(mark);
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
