# Round-4: 128-channel 3x3 conv with K-split waves (32 output channels x half the input
# channels per wave): numerics, per-layer timing, ResNet bench
set -o pipefail
mkdir -p gpurun_out/c128
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_cnn_gpu.py -k "28-28-128-128 or 28-28-128" > gpurun_out/c128/t.log 2>&1 || exit 1
ONLY=layer2.1,layer2.2,layer1.1 timeout -k 10 200 python -u tools/probes/resnet_layers.py > gpurun_out/c128/layers.jsonl 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py tests/test_resnet_gpu.py > gpurun_out/c128/t2.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/c128/resnet_$r.json 2>/dev/null || exit 1
done
echo done
