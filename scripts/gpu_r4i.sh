#!/bin/bash
# Async PS after the background sender: tests, breakdown, cluster benches (TCP 2 / 8, GPU store).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4i}; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== ps tests"
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_ps.log" 2>&1 || { tail -30 "$OUT/pytest_ps.log"; exit 1; }
tail -1 "$OUT/pytest_ps.log"
echo "== ps"
for rep in 1 2; do
timeout -k 10 200 python tools/probes/ps_worker_breakdown.py --mode pipelined > "$OUT/ps_breakdown_$rep.json" 2>&1 || exit 1
tail -1 "$OUT/ps_breakdown_$rep.json"
done
timeout -k 10 200 python tools/bench_ps_async.py --num_workers 2 --steps 40000 > "$OUT/ps_async_w2.json" 2>/dev/null || exit 1
timeout -k 10 200 python tools/bench_ps_async.py --num_workers 8 --steps 40000 > "$OUT/ps_async_w8.json" 2>/dev/null || exit 1
timeout -k 10 200 python tools/bench_ps_async.py --num_workers 2 --steps 40000 --ps_device gpu > "$OUT/ps_async_gpu_w2.json" 2>/dev/null || exit 1
cut -c 1-170 "$OUT/ps_async_w2.json" "$OUT/ps_async_w8.json" "$OUT/ps_async_gpu_w2.json"
