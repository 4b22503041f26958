# ResNet-50 kernel profile + per-layer conv timings (round 4, after the BatchNorm fusions)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
OUT=gpurun_out/rprof4
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cnn_gpu.py tests/test_resnet_gpu.py > "$OUT/t.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rprof" -o run -- python "$R/bench.py" --model resnet50 --steps 6 --warmup 3 > "$OUT/rprof.log" 2>&1 || exit 1
python "$R/tools/prof_summary.py" "$OUT/rprof/run_kernel_stats.csv" > "$OUT/resnet_kernel_stats.txt" || exit 1
python "$R/tools/trace_by_shape.py" "$OUT/rprof/run_kernel_trace.csv" 70 > "$OUT/resnet_kernel_shapes.txt" || exit 1
python "$R/tools/trace_gaps.py" "$OUT/rprof/run_kernel_trace.csv" --window sgd_momentum > "$OUT/resnet_gaps.txt" || exit 1
rm -f "$OUT"/rprof/*trace.csv
timeout -k 10 240 python -u tools/probes/resnet_layers.py > "$OUT/resnet_layers.jsonl" 2>&1 || exit 1
tail -1 "$OUT/resnet_layers.jsonl"
echo done
