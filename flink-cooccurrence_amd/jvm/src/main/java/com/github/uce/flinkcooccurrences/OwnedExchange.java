package com.github.uce.flinkcooccurrences;

import java.io.IOException;
import java.nio.file.Files;
import java.nio.file.Path;
import java.nio.file.Paths;
import java.nio.file.StandardCopyOption;
import java.util.Arrays;

/**
 * The per-subtask side of the p > 1 one-window exchange shared by GpuOwnedCooccurrenceRowsOperator and
 * GpuOwnedCooccurrenceTopKOperator: the communicator rendezvous, the window the p subtasks fire together,
 * and the buffered keyBy(user) shard as CSR.
 *
 * <p><b>Communicator id per attempt.</b> An RCCL id is single-use and its bootstrap root lives in the process
 * that created it.  Subtask 0 creates it in open() -- inside the TaskManager, once per execution attempt -- and
 * publishes it as {@code <rendezvousDir>/<jobId>-<attempt>.commid} (written to a temporary name, then renamed,
 * so a reader never sees a partial id); subtasks 1..p-1 poll for that file and fail the task after
 * {@link #RENDEZVOUS_TIMEOUT_MS} (IllegalStateException) instead of hanging in the communicator's init.  The 8
 * GPUs of a node share one TaskManager host, so a node-local directory serves; a restarted attempt rendezvous
 * under its own attempt number with a fresh id.
 *
 * <p><b>Late records.</b> As in NonSampledUserInteractionCounterOneInputStreamOperator.processElement (:84-91), a
 * record whose timestamp is at or below this subtask's current watermark is dropped and counted in the
 * {@code UserInteractionCounterLateElements} accumulator ({@link #add} returns false); the watermark is the
 * subtask's own, as the reference's timerService.currentWatermark() is.
 *
 * <p><b>One window, agreed.</b> Flink does not hand every subtask the same watermarks: each subtask's is the
 * minimum over its own input channels, which arrive in their own order.  So what fires is decided from
 * all-gathered state only.  An agreement step all-gathers (cooc_comm_allgather_i64) every subtask's watermark and
 * window start (Long.MIN_VALUE while it holds no record); {@code agreed} becomes the minimum watermark -- a record
 * of a window ending at or below it is late on every subtask -- and the window fires on EVERY subtask once its
 * end is at or below {@code agreed} (a subtask without records joins the same collectives with an empty shard).
 * A subtask runs steps while its own watermark is ahead of {@code agreed}, waiting in the collective for the
 * others to catch up; both the condition and the outcome depend only on all-gathered values and on watermarks
 * that only grow, so every subtask runs the same sequence of collectives.  Records of two different windows
 * fail every subtask alike (IllegalStateException).  Multi-window streams use the library's per-window exchange
 * instead (GpuCooccurrenceJob.topKStreamOwned, the same agreement inside cooc_op_process_watermark), which shares
 * {@link #rendezvous}.
 */
final class OwnedExchange {

  static final long RENDEZVOUS_TIMEOUT_MS = 120_000;

  private final long windowSizeMs;
  private final long handle;
  private final int world;
  private int buffered;
  private int[] users = new int[1 << 16];
  private int[] items = new int[1 << 16];
  private long windowStart = Long.MIN_VALUE;
  private long watermark = Long.MIN_VALUE;  // this subtask's own (timerService.currentWatermark())
  private long agreed = Long.MIN_VALUE;     // the minimum watermark over the subtasks at the last step
  private boolean fired;

  OwnedExchange(long handle, long windowSizeMs, int world) {
    this.handle = handle;
    this.windowSizeMs = windowSizeMs;
    this.world = world;
  }

  /** The communicator id of this attempt: created by subtask 0, read by the others (see the class comment). */
  static byte[] rendezvous(String dir, String jobId, int attempt, int subtask) throws IOException, InterruptedException {
    final Path path = Paths.get(dir, jobId + "-" + attempt + ".commid");
    if (subtask == 0) {
      final byte[] id = CoocNative.commUniqueId();
      final Path tmp = Paths.get(dir, jobId + "-" + attempt + ".commid.tmp");
      Files.write(tmp, id);
      Files.move(tmp, path, StandardCopyOption.ATOMIC_MOVE, StandardCopyOption.REPLACE_EXISTING);
      return id;
    }
    final long deadline = System.currentTimeMillis() + RENDEZVOUS_TIMEOUT_MS;
    while (!Files.exists(path)) {
      if (System.currentTimeMillis() > deadline) {
        throw new IllegalStateException("no communicator id from subtask 0 at " + path + " after "
            + RENDEZVOUS_TIMEOUT_MS + " ms");
      }
      Thread.sleep(50);
    }
    return Files.readAllBytes(path);
  }

  /**
   * processElement: false for a late record (ts at or below this subtask's watermark: dropped, the caller counts
   * it, NonSampled...java:89-91); otherwise the record joins the shard, and it must fall in the shard's window
   * (offset 0 tumbling).
   */
  boolean add(int user, int item, long ts) {
    if (ts <= watermark) {
      return false;
    }
    final long start = ts - Math.floorMod(ts, windowSizeMs);
    if (windowStart == Long.MIN_VALUE) {
      windowStart = start;
    } else if (start != windowStart || fired) {
      throw new IllegalStateException("the owned-rows operators serve one window; record at " + ts);
    }
    if (buffered == users.length) {
      users = Arrays.copyOf(users, 2 * buffered);
      items = Arrays.copyOf(items, 2 * buffered);
    }
    users[buffered] = user;
    items[buffered] = item;
    buffered++;
    return true;
  }

  /**
   * processWatermark: the maxTimestamp of the window every subtask fires now, or Long.MIN_VALUE.  Collective (see
   * the class comment): it may wait for the other subtasks' watermarks to catch up with this one.
   */
  long fireAt(long mark) {
    if (mark > watermark) {
      watermark = mark;
    }
    while (!fired && watermark > agreed) {
      long wmin = Long.MAX_VALUE;
      for (long w : CoocNative.commAllGather(handle, watermark, world)) {
        wmin = Math.min(wmin, w);
      }
      long start = Long.MIN_VALUE;
      for (long s : CoocNative.commAllGather(handle, windowStart, world)) {
        if (s == Long.MIN_VALUE) {
          continue;
        }
        if (start != Long.MIN_VALUE && s != start) {
          throw new IllegalStateException("subtasks hold records of two windows: " + start + " and " + s);
        }
        start = s;
      }
      agreed = Math.max(agreed, wmin);
      if (start != Long.MIN_VALUE && start + windowSizeMs - 1 <= agreed) {
        fired = true;
        return start + windowSizeMs - 1;
      }
    }
    return Long.MIN_VALUE;
  }

  /** The shard as CSR (users ascending, each user's items in arrival order) through countOwned. */
  long[] countOwned() {
    final Integer[] idx = new Integer[buffered];
    for (int i = 0; i < buffered; i++) {
      idx[i] = i;
    }
    final int[] u = users;
    Arrays.sort(idx, (x, y) -> u[x] != u[y] ? Integer.compare(u[x], u[y]) : Integer.compare(x, y));
    final int[] ordered = new int[buffered];
    int nUsers = 0;
    for (int i = 0; i < buffered; i++) {
      ordered[i] = items[idx[i]];
      if (i == 0 || u[idx[i]] != u[idx[i - 1]]) {
        nUsers++;
      }
    }
    final long[] userPtr = new long[nUsers + 1];
    for (int i = 0, k = 0; i < buffered; i++) {
      if (i > 0 && u[idx[i]] != u[idx[i - 1]]) {
        userPtr[++k] = i;
      }
    }
    userPtr[nUsers] = buffered;
    buffered = 0;
    users = new int[1];
    items = new int[1];
    return CoocNative.countOwned(handle, userPtr, ordered);  // {nnz, observed, rows, job observed}
  }
}
