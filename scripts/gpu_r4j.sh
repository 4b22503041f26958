#!/bin/bash
# 16-byte LL pair exchange: engine tests first, then the split A/B (0 = 8-byte by the K-split-0
# wave, 1 = 16-byte pairs over both waves), then the trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4j}; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== engine tests"
timeout -k 10 700 python -u -m pytest tests/test_xgmi_sim_gpu.py "tests/test_xgmi_gpu.py::test_fused_mlp_exchange_matches_allreduce_engine" "tests/test_xgmi_gpu.py::test_factor_mlp_exchange_matches_allreduce_engine" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_engines.log" 2>&1 || { tail -30 "$OUT/pytest_engines.log"; exit 1; }
tail -1 "$OUT/pytest_engines.log"
for rep in 1 2; do
  for sp in ${SPLITS:-0 1}; do
    DTFX_XG_SPLIT=$sp timeout -k 10 200 python tools/probes/engine_local_cost.py > "$OUT/local_cost_split${sp}_$rep.json" 2>&1 || { tail -5 "$OUT/local_cost_split${sp}_$rep.json"; exit 1; }
    echo "split=$sp rep=$rep $(python -c "import json,sys; t=json.loads(open(sys.argv[1]).read().split(chr(10),1)[1]); print(t['single_gpu_2launch_us'], {w: (t[w]['fused2'], t[w]['fused2x']) for w in ('world2','world4','world8')})" "$OUT/local_cost_split${sp}_$rep.json")"
  done
done
timeout -k 10 200 python tools/probes/engine_trace.py > "$OUT/engine_trace.json" 2>&1 || { tail -5 "$OUT/engine_trace.json"; exit 1; }
python - "$OUT/engine_trace.json" <<'PY'
import json, sys
t = json.loads(open(sys.argv[1]).read().split("\n", 1)[1])
for w in ("world2", "world4", "world8"):
    for e, v in t[w].items():
        print(w, e, {k: v[k] for k in v if k.startswith(("exchange", "small", "w1_span", "span"))})
PY
