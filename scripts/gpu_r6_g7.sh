#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/g7
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_streaming_multiproc.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
echo "tests ok"
timeout -k 10 300 python bench.py --config c4 > $O/c4.json 2> $O/c4.err || { echo "c4 failed"; tail -20 $O/c4.err; exit 1; }
timeout -k 10 300 python bench.py --config c2 --steps 10 > $O/c2.json 2> $O/c2.err || { echo "c2 failed"; tail -20 $O/c2.err; exit 1; }
python3 - <<'PY'
import json
for f in ["c4", "c2"]:
    d = json.loads(open(f"gpurun_out/g7/{f}.json").read().strip().splitlines()[-1])
    print(f, "value %.3g" % d["value"], "ms/step %.2f" % d["ms_per_step"], "frac", d["roofline"]["frac"], d.get("roofline_lds", {}).get("frac"), d["config"].get("window_latency_ms"))
PY
