#!/bin/bash
# End-of-round check of the tree as the driver runs it: smoke, the whole GPU tier, the default
# bench (driver-sized) -- each under its own limit, stopping at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/final; mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python bench.py > $OUT/bench_default.json 2>&1 || exit 1
tail -1 $OUT/bench_default.json | cut -c 1-200
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_k20.json 2>&1 || exit 1
tail -1 $OUT/bench_k20.json | cut -c 1-200
