#!/bin/bash
# Exchange-engine tests + trace/local cost, then the async-PS worker.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4g}; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== engine tests"
timeout -k 10 700 python -u -m pytest tests/test_xgmi_sim_gpu.py "tests/test_xgmi_gpu.py::test_fused_mlp_exchange_matches_allreduce_engine" "tests/test_xgmi_gpu.py::test_factor_mlp_exchange_matches_allreduce_engine" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_engines.log" 2>&1 || { tail -30 "$OUT/pytest_engines.log"; exit 1; }
tail -1 "$OUT/pytest_engines.log"
echo "== engine trace"
timeout -k 10 200 python tools/probes/engine_trace.py > "$OUT/engine_trace.json" 2>&1 || { tail -5 "$OUT/engine_trace.json"; exit 1; }
timeout -k 10 200 python tools/probes/engine_local_cost.py > "$OUT/engine_local_cost.json" 2>&1 || { tail -5 "$OUT/engine_local_cost.json"; exit 1; }
grep -E "span|small|world|exchange" "$OUT/engine_trace.json" | tr -d '\n ' | sed 's/"world/\n"world/g'; echo
tr -d '\n ' < "$OUT/engine_local_cost.json"; echo
TAG=${TAG:-r4g} bash scripts/gpu_r4f.sh
