# Round-4: BERT-base kernel profile with the final defaults
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=$(pwd); OUT=$R/gpurun_out/bprof_final; mkdir -p $OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p" -o run -- python "$R/bench.py" --model bert --steps 6 --warmup 3 > "$OUT/p.log" 2>&1 || exit 1
python "$R/tools/prof_summary.py" "$OUT/p/run_kernel_stats.csv" > "$OUT/bert_kernel_stats.txt"
python "$R/tools/trace_by_shape.py" "$OUT/p/run_kernel_trace.csv" 40 > "$OUT/bert_kernel_shapes.txt"
python "$R/tools/trace_gaps.py" "$OUT/p/run_kernel_trace.csv" > "$OUT/bert_gaps.txt" 2>&1 || true
rm -f "$OUT"/p/*trace.csv
echo done
