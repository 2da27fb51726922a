import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as g
pkg = g.load_package()
from flink_cooccurrence_amd import datagen
M = int(sys.argv[1]) if len(sys.argv) > 1 else 40_500
d = datagen.config_c1(seed=5, U=1500, M=M, mean=20.0)
users, items, ts = datagen.to_records(d["user_ptr"], d["items"], d["ts"])
op = pkg.NonSampledUserInteractionCounterOneInputStreamOperator(1, "SECONDS", n_items=M, top_k=10)
t0 = time.time(); n = 0
for lo in range(0, len(users), 5000):
    sl = slice(lo, lo + 5000)
    op.process_elements(users[sl], items[sl], ts[sl])
    print("elements", lo, time.time() - t0, flush=True)
    n += len(op.process_watermark(int(ts[sl][-1]) - 1))
    print("windows", n, time.time() - t0, flush=True)
