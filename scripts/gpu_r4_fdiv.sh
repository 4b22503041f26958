# Round-4: conv GEMM tap decode by float reciprocals -- numerics, layer3/4 conv timings, ResNet
set -o pipefail
mkdir -p gpurun_out/fdiv
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py tests/test_resnet_gpu.py tests/test_bf16_gpu.py > gpurun_out/fdiv/t.log 2>&1 || exit 1
ONLY=layer3.0,layer3.1,layer4.0,layer4.1,layer2.0 timeout -k 10 300 python -u tools/probes/resnet_layers.py > gpurun_out/fdiv/layers.jsonl 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/fdiv/resnet_$r.json 2>/dev/null || exit 1
done
echo done
