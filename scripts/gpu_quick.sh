#!/bin/bash
# Quick GPU check: driver smoke, the GPU test tier, the driver-sized MLP bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/quick; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
echo "== tests"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
echo "== bench"
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > "$OUT/bench_k20.json" 2>&1 || { tail -5 "$OUT/bench_k20.json"; exit 1; }
tail -1 "$OUT/bench_k20.json" | cut -c 1-200
