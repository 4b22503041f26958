# kernel stats of the ResNet step with / without the compact stride-2 downsample gradient
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=$(pwd); OUT=$R/gpurun_out/dscp; mkdir -p $OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/on" -o run -- python "$R/bench.py" --model resnet50 --steps 6 --warmup 3 > "$OUT/on.log" 2>&1 || exit 1
DTFX_DS_COMPACT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/off" -o run -- python "$R/bench.py" --model resnet50 --steps 6 --warmup 3 > "$OUT/off.log" 2>&1 || exit 1
python "$R/tools/trace_by_shape.py" "$OUT/on/run_kernel_trace.csv" 60 > "$OUT/on_shapes.txt"
python "$R/tools/trace_by_shape.py" "$OUT/off/run_kernel_trace.csv" 60 > "$OUT/off_shapes.txt"
rm -f "$OUT"/on/*trace.csv "$OUT"/off/*trace.csv
echo done
