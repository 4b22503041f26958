#!/bin/bash
# BERT-base step timeline: rocprofv3 kernel trace (timestamps per kernel, per queue).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT=$R/gpurun_out/${TAG:-btrace}; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- python "$R/bench.py" --model bert --steps 6 --warmup 3 > "$OUT/bprof.log" 2>&1 || { tail -20 "$OUT/bprof.log"; exit 1; }
tail -1 "$OUT/bprof.log" | cut -c 1-200
python "$R/tools/trace_gaps.py" "$OUT/prof/run_kernel_trace.csv" --window adam_mixed > "$OUT/gaps.txt" 2>&1 || true
head -40 "$OUT/gaps.txt"
gzip -f "$OUT/prof/run_kernel_trace.csv"
