# 3x3 weight gradients on the 8-phase tile: tests, per-layer timings and interleaved A/B
set -o pipefail
mkdir -p gpurun_out/wg8
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cnn_gpu.py tests/test_resnet_gpu.py > gpurun_out/wg8/t.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/probes/resnet_layers.py > gpurun_out/wg8/layers_on.jsonl 2>&1 || exit 1
DTFX_CONV_WGRAD_PH8=0 timeout -k 10 240 python -u tools/probes/resnet_layers.py > gpurun_out/wg8/layers_off.jsonl 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/wg8/on_$r.json 2>/dev/null || exit 1
  DTFX_CONV_WGRAD_PH8=0 timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/wg8/off_$r.json 2>/dev/null || exit 1
done
echo done
