"""Debug harness: one small large-universe (n_items >= 40,320) window through cooc_count_host."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__
pkg = __graft_entry__.load_package()
from flink_cooccurrence_amd import datagen
from oracle import oracle
U, M, mean = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])
up, it = datagen.small_log(4, U, M, mean, replacement=True)
print("log", U, M, len(it), flush=True)
t0 = time.time()
with pkg.CooccurrenceCore(n_items=M) as core:
    got = core.count(up, it)
print("counted", time.time() - t0, flush=True)
rp, cols, data, rowsums, observed = oracle.closed_form(up, it, M)
print("observed", got.observed == observed, "rowptr", np.array_equal(got.row_ptr, rp), "cols", np.array_equal(got.cols, cols),
      "cnt", np.array_equal(got.cnt.astype(np.int64), data), "rowsum", np.array_equal(got.rowsum, rowsums), flush=True)
