#!/bin/bash
# BERT-base: GPU tests for the transformer kernels, bench, rocprofv3 kernel trace + stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT=$R/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_transformer_gpu.py tests/test_bf16_gpu.py tests/test_bert_gpu.py ${EXTRA_TESTS:-} > "$OUT/t_bert.log" 2>&1 \
    || { echo FAIL tests; tail -30 "$OUT/t_bert.log"; exit 1; }
  tail -3 "$OUT/t_bert.log"
fi
timeout -k 10 300 python bench.py --model bert ${BENCH_ARGS:-} > "$OUT/bench_bert.log" 2>&1 || { echo FAIL bench; tail -20 "$OUT/bench_bert.log"; exit 1; }
tail -1 "$OUT/bench_bert.log"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bprof" -o run -- \
  python "$R/bench.py" --model bert --steps 6 --warmup 3 ${BENCH_ARGS:-} > "$OUT/bprof.log" 2>&1 || { echo FAIL prof; tail -20 "$OUT/bprof.log"; exit 1; }
python "$R/tools/prof_summary.py" "$OUT/bprof/run_kernel_stats.csv" > "$OUT/bprof_summary.txt" 2>&1; head -30 "$OUT/bprof_summary.txt"
python "$R/tools/trace_by_shape.py" "$OUT/bprof/run_kernel_trace.csv" > "$OUT/bprof_shapes.txt" 2>&1; head -40 "$OUT/bprof_shapes.txt"
