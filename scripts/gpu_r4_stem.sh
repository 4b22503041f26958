# Round-4: stem forward on 16 x 16 tiles (4 rows per wave, parity-split patch): numerics,
# stem layer timing, ResNet bench
set -o pipefail
mkdir -p gpurun_out/stem
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py tests/test_resnet_gpu.py > gpurun_out/stem/t.log 2>&1 || exit 1
ONLY=conv1 timeout -k 10 200 python -u tools/probes/resnet_layers.py > gpurun_out/stem/layers.jsonl 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/stem/resnet_$r.json 2>/dev/null || exit 1
done
echo done
