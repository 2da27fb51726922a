package com.github.uce.flinkcooccurrences;

import it.unimi.dsi.fastutil.ints.Int2ShortMap;
import it.unimi.dsi.fastutil.ints.Int2ShortOpenHashMap;
import java.util.concurrent.TimeUnit;
import org.apache.flink.api.common.functions.ReduceFunction;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.api.java.tuple.Tuple3;
import org.apache.flink.streaming.api.datastream.DataStream;
import org.apache.flink.streaming.api.datastream.SingleOutputStreamOperator;
import org.apache.flink.streaming.api.windowing.assigners.TumblingEventTimeWindows;
import org.apache.flink.streaming.api.windowing.time.Time;

/**
 * The {@code --skip-cuts} graph of FlinkCooccurrences.main with the GPU operator: replaces
 * FlinkCooccurrences.java:65-74 (the pair emitter) and :135-157 (ItemRowAggregator and RowSumAggregator
 * windows) and returns the same rescorer wiring as :162-167.  In main:
 * <pre>
 *   DataStream&lt;Tuple2&lt;Integer, IntDoublePriorityQueue&gt;&gt; topKStream = skipCuts
 *       ? GpuCooccurrenceJob.topK(interactionStream, windowSize, windowUnit, nItems, devices, configuration.getTopK(),
 *                                 gpuRescore)
 *       : ...the reference's sampled graph...;
 * </pre>
 * Uncompiled here (no JDK); see GpuNonSampledCooccurrenceRowsOperator.
 */
final class GpuCooccurrenceJob {

  private GpuCooccurrenceJob() {
  }

  static DataStream<Tuple2<Integer, IntDoublePriorityQueue>> topK(
      DataStream<Tuple3<Integer, Integer, Long>> interactionStream, int windowSize, TimeUnit windowUnit, int nItems,
      int[] devices, short topK) {
    return topK(interactionStream, windowSize, windowUnit, nItems, devices, topK, false);
  }

  /**
   * gpuRescore: the rescorer runs on the device too (GpuNonSampledCooccurrenceTopKOperator replaces
   * FlinkCooccurrences.java:65-74 AND :135-167); one subtask holds every user and the global rows.
   * Otherwise the rows operator feeds the reference's ItemRowRescorerTwoInputStreamOperator.
   */
  static DataStream<Tuple2<Integer, IntDoublePriorityQueue>> topK(
      DataStream<Tuple3<Integer, Integer, Long>> interactionStream, int windowSize, TimeUnit windowUnit, int nItems,
      int[] devices, short topK, boolean gpuRescore) {
    if (gpuRescore) {
      return interactionStream
          .keyBy(0)
          .transform(
              "GpuNonSampledCooccurrenceTopK (" + windowSize + " " + windowUnit + ", top " + topK + ")",
              GpuNonSampledCooccurrenceTopKOperator.getOutputType(),
              new GpuNonSampledCooccurrenceTopKOperator(windowSize, windowUnit, nItems, devices, topK))
          .setParallelism(1);
    }
    final SingleOutputStreamOperator<Void> counter = interactionStream
        .keyBy(0)
        .transform(
            "GpuNonSampledCooccurrenceRows (" + windowSize + " " + windowUnit + ")",
            GpuNonSampledCooccurrenceRowsOperator.getOutputType(),
            new GpuNonSampledCooccurrenceRowsOperator(windowSize, windowUnit, nItems, devices));
    DataStream<Tuple2<Integer, Int2ShortOpenHashMap>> rowStream =
        counter.getSideOutput(GpuNonSampledCooccurrenceRowsOperator.ROWS_TAG);
    DataStream<Tuple2<Integer, Integer>> rowSumStream =
        counter.getSideOutput(GpuNonSampledCooccurrenceRowsOperator.ROW_SUM_TAG);
    if (counter.getParallelism() > 1) {
      // every subtask holds a user shard: sum its partial rows / int row sums per item and window (the
      // reference's keyBy(item) windows, FlinkCooccurrences.java:138-157, over p records per row)
      rowStream = rowStream.keyBy(0)
          .window(TumblingEventTimeWindows.of(Time.of(windowSize, windowUnit)))
          .reduce(new ItemRowMerge())
          .name("ItemRowMerge");
      rowSumStream = rowSumStream.keyBy(0)
          .window(TumblingEventTimeWindows.of(Time.of(windowSize, windowUnit)))
          .reduce(new IntSum())
          .filter(t -> t.f1 != 0)  // RowSumAggregator.java:66
          .name("RowSumMerge");
    }
    return rowStream
        .keyBy(0).connect(rowSumStream.broadcast())
        .transform(
            "ItemRowRescorer",
            ItemRowRescorerTwoInputStreamOperator.getOutputType(),
            new ItemRowRescorerTwoInputStreamOperator(topK));
  }

  /**
   * p > 1 subtasks, a multi-window stream (any n_items): the keyBy(item) merge of partial rows replaced by
   * the library's exchange per window (cooc.h, cooc_finish_window across GPUs).  Each subtask keeps its users'
   * histories and the global rows it owns resident; gpuRescore: GpuNonSampledCooccurrenceTopKOperator rescores
   * the owned rows on the device at parallelism p; otherwise the rows operator's complete owned rows and their
   * job-wide row sums feed the reference's rescorer with no ItemRowMerge / RowSumMerge windows.
   */
  static DataStream<Tuple2<Integer, IntDoublePriorityQueue>> topKStreamOwned(
      DataStream<Tuple3<Integer, Integer, Long>> interactionStream, int windowSize, TimeUnit windowUnit, int nItems,
      int[] devices, short topK, int parallelism, String rendezvousDir, boolean gpuRescore) {
    if (gpuRescore) {
      return interactionStream
          .keyBy(0)
          .transform(
              "GpuNonSampledCooccurrenceTopK (" + windowSize + " " + windowUnit + ", top " + topK + ", "
                  + parallelism + " GPUs)",
              GpuNonSampledCooccurrenceTopKOperator.getOutputType(),
              new GpuNonSampledCooccurrenceTopKOperator(windowSize, windowUnit, nItems, devices, topK, rendezvousDir))
          .setParallelism(parallelism);
    }
    final SingleOutputStreamOperator<Void> counter = interactionStream
        .keyBy(0)
        .transform(
            "GpuNonSampledCooccurrenceRows (" + windowSize + " " + windowUnit + ", " + parallelism + " GPUs)",
            GpuNonSampledCooccurrenceRowsOperator.getOutputType(),
            new GpuNonSampledCooccurrenceRowsOperator(windowSize, windowUnit, nItems, devices, rendezvousDir))
        .setParallelism(parallelism);
    return counter.getSideOutput(GpuNonSampledCooccurrenceRowsOperator.ROWS_TAG)
        .keyBy(0).connect(counter.getSideOutput(GpuNonSampledCooccurrenceRowsOperator.ROW_SUM_TAG).broadcast())
        .transform(
            "ItemRowRescorer",
            ItemRowRescorerTwoInputStreamOperator.getOutputType(),
            new ItemRowRescorerTwoInputStreamOperator(topK));
  }

  /**
   * p > 1 subtasks, one window (the C3 / C5 configs): the keyBy(item) merge of partial rows replaced by the
   * library's exchange over RCCL.  gpuRescore: GpuOwnedCooccurrenceTopKOperator rescores the owned rows on the
   * device too and emits the rescorer's records itself (C5 never rescores on the JVM); otherwise
   * GpuOwnedCooccurrenceRowsOperator's complete owned rows feed the reference's rescorer with no ItemRowMerge /
   * RowSumMerge windows.  Each execution attempt's communicator id is created by subtask 0 in open() and handed
   * over through rendezvousDir (a directory every subtask of the node can read, OwnedExchange).
   */
  static DataStream<Tuple2<Integer, IntDoublePriorityQueue>> topKOwned(
      DataStream<Tuple3<Integer, Integer, Long>> interactionStream, int windowSize, TimeUnit windowUnit, int nItems,
      int[] devices, short topK, int parallelism, String rendezvousDir, boolean gpuRescore) {
    if (gpuRescore) {
      return interactionStream
          .keyBy(0)
          .transform(
              "GpuOwnedCooccurrenceTopK (" + windowSize + " " + windowUnit + ", top " + topK + ", " + parallelism
                  + " GPUs)",
              GpuNonSampledCooccurrenceTopKOperator.getOutputType(),
              new GpuOwnedCooccurrenceTopKOperator(windowSize, windowUnit, nItems, devices, topK, rendezvousDir))
          .setParallelism(parallelism);
    }
    final SingleOutputStreamOperator<Void> counter = interactionStream
        .keyBy(0)
        .transform(
            "GpuOwnedCooccurrenceRows (" + windowSize + " " + windowUnit + ", " + parallelism + " GPUs)",
            GpuNonSampledCooccurrenceRowsOperator.getOutputType(),
            new GpuOwnedCooccurrenceRowsOperator(windowSize, windowUnit, nItems, devices, rendezvousDir))
        .setParallelism(parallelism);
    return counter.getSideOutput(GpuNonSampledCooccurrenceRowsOperator.ROWS_TAG)
        .keyBy(0).connect(counter.getSideOutput(GpuNonSampledCooccurrenceRowsOperator.ROW_SUM_TAG).broadcast())
        .transform(
            "ItemRowRescorer",
            ItemRowRescorerTwoInputStreamOperator.getOutputType(),
            new ItemRowRescorerTwoInputStreamOperator(topK));
  }

  /** Int2ShortOpenHashMap.addTo of every entry (short arithmetic wraps, ItemRowAggregator.java:29). */
  static final class ItemRowMerge implements ReduceFunction<Tuple2<Integer, Int2ShortOpenHashMap>> {
    private static final long serialVersionUID = 1L;

    @Override
    public Tuple2<Integer, Int2ShortOpenHashMap> reduce(Tuple2<Integer, Int2ShortOpenHashMap> a,
        Tuple2<Integer, Int2ShortOpenHashMap> b) {
      for (Int2ShortMap.Entry e : b.f1.int2ShortEntrySet()) {
        a.f1.addTo(e.getIntKey(), e.getShortValue());
      }
      return a;
    }
  }

  /** Java int sum of the partial row-sum deltas (RowSumAggregator.java:25-27 wraps the same way). */
  static final class IntSum implements ReduceFunction<Tuple2<Integer, Integer>> {
    private static final long serialVersionUID = 1L;

    @Override
    public Tuple2<Integer, Integer> reduce(Tuple2<Integer, Integer> a, Tuple2<Integer, Integer> b) {
      return Tuple2.of(a.f0, a.f1 + b.f1);
    }
  }
}
