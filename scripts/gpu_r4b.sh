#!/bin/bash
# MLP exchange engines: simulated-peer + two-process tests, the per-phase trace, local cost.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4b}; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== tests"
timeout -k 10 700 python -u -m pytest tests/test_xgmi_sim_gpu.py "tests/test_xgmi_gpu.py::test_fused_mlp_exchange_matches_allreduce_engine" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
echo "== engine trace"
timeout -k 10 200 python tools/probes/engine_trace.py > "$OUT/engine_trace.json" 2>&1 || { tail -5 "$OUT/engine_trace.json"; exit 1; }
timeout -k 10 200 python tools/probes/engine_local_cost.py > "$OUT/engine_local_cost.json" 2>&1 || { tail -5 "$OUT/engine_local_cost.json"; exit 1; }
python - "$OUT" <<'PY'
import json, sys
o = sys.argv[1]
t = json.loads(open(o + "/engine_trace.json").read().split("\n", 1)[1] if open(o + "/engine_trace.json").read().startswith("/") else open(o + "/engine_trace.json").read())
for w in ("world2", "world4", "world8"):
    for e, v in t[w].items():
        print(w, e, "exchange", v.get("exchange"), "hop1", v.get("hop1"), "hop2", v.get("hop2"), "span", v.get("span_us"))
PY
cat "$OUT/engine_local_cost.json"
