#!/bin/bash
# Engine trace (small blocks separated) + async-PS worker (native step, staged batch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4f}; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== ps tests"
timeout -k 10 600 python -u -m pytest ${PS_TESTS:-tests/test_train_gpu.py} -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
echo "== ps"
timeout -k 10 200 python tools/probes/ps_worker_breakdown.py --mode pipelined > "$OUT/ps_breakdown.json" 2>&1 || exit 1
tail -1 "$OUT/ps_breakdown.json"
timeout -k 10 200 python tools/bench_ps_async.py --num_workers 2 --steps 40000 > "$OUT/ps_async_w2.json" 2>/dev/null || exit 1
cut -c 1-200 "$OUT/ps_async_w2.json"
echo "== engine trace"
timeout -k 10 200 python tools/probes/engine_trace.py > "$OUT/engine_trace.json" 2>&1 || { tail -5 "$OUT/engine_trace.json"; exit 1; }
grep -E "span|small|world" "$OUT/engine_trace.json" | tr -d '\n' | sed 's/"world/\n"world/g'; echo
