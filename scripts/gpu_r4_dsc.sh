# Round-4 A/B: stride-2 downsample data gradient kept compact (read by conv1's wide dgrad as a
# stride-2 residual) vs materialised at full resolution; interleaved on one box
set -o pipefail
mkdir -p gpurun_out/dsc
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py tests/test_resnet_gpu.py > gpurun_out/dsc/t.log 2>&1 || exit 1
timeout -k 10 200 python tools/probes/ds_compact_gemm.py > gpurun_out/dsc/gemm.jsonl 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/dsc/on_$r.json 2>/dev/null || exit 1
  DTFX_DS_COMPACT=0 timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/dsc/off_$r.json 2>/dev/null || exit 1
done
echo done
