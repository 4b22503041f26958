#!/bin/bash
# A/B of the exchange splits (DTFX_XG_SPLIT bit 0: W1 slices over both K-split waves, bit 1:
# small parameters over two waves), interleaved, same box; then the engine tests; then PS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4h}; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
  for sp in 0 1 3; do
    DTFX_XG_SPLIT=$sp timeout -k 10 200 python tools/probes/engine_local_cost.py > "$OUT/local_cost_split${sp}_$rep.json" 2>&1 || { tail -5 "$OUT/local_cost_split${sp}_$rep.json"; exit 1; }
    echo "split=$sp rep=$rep $(python -c "import json,sys; t=json.loads(open(sys.argv[1]).read().split(chr(10),1)[1]); print(t['single_gpu_2launch_us'], {w: (t[w]['fused2'], t[w]['fused2x']) for w in ('world2','world4','world8')})" "$OUT/local_cost_split${sp}_$rep.json")"
  done
done
echo "== engine tests"
timeout -k 10 700 python -u -m pytest tests/test_xgmi_sim_gpu.py "tests/test_xgmi_gpu.py::test_fused_mlp_exchange_matches_allreduce_engine" "tests/test_xgmi_gpu.py::test_factor_mlp_exchange_matches_allreduce_engine" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_engines.log" 2>&1 || { tail -30 "$OUT/pytest_engines.log"; exit 1; }
tail -1 "$OUT/pytest_engines.log"
echo "== ps tests"
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_ps.log" 2>&1 || { tail -30 "$OUT/pytest_ps.log"; exit 1; }
tail -1 "$OUT/pytest_ps.log"
echo "== ps"
DTFX_PS_NO_ZERO_COPY=1 timeout -k 10 200 python tools/probes/ps_worker_breakdown.py --mode pipelined > "$OUT/ps_breakdown_copies.json" 2>&1 || exit 1
timeout -k 10 200 python tools/probes/ps_worker_breakdown.py --mode pipelined > "$OUT/ps_breakdown.json" 2>&1 || exit 1
tail -1 "$OUT/ps_breakdown_copies.json"; tail -1 "$OUT/ps_breakdown.json"
timeout -k 10 200 python tools/bench_ps_async.py --num_workers 2 --steps 40000 > "$OUT/ps_async_w2.json" 2>/dev/null || exit 1
cut -c 1-200 "$OUT/ps_async_w2.json"
