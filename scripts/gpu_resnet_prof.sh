#!/bin/bash
# ResNet-50: rocprofv3 kernel trace of a short run, grouped by kernel and grid.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT=$R/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rprof" -o run -- \
  python "$R/bench.py" --model resnet50 --steps 4 --warmup 2 > "$OUT/rprof.log" 2>&1 || { echo FAIL prof; tail -20 "$OUT/rprof.log"; exit 1; }
python "$R/tools/trace_by_shape.py" "$OUT/rprof/run_kernel_trace.csv" 60 > "$OUT/rprof_shapes.txt" 2>&1
python "$R/tools/prof_summary.py" "$OUT/rprof/run_kernel_stats.csv" > "$OUT/rprof_summary.txt" 2>&1
head -30 "$OUT/rprof_summary.txt"; head -62 "$OUT/rprof_shapes.txt"
