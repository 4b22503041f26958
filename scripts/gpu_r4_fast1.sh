# Round-4: 1x1 / stride-1 conv GEMMs on the 8-phase tile with their own staging instantiation
# (cfg 7) -- numerics, per-layer timings, ResNet A/B (DTFX_CONV_F1=0: the general staging)
set -o pipefail
mkdir -p gpurun_out/fast1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py tests/test_resnet_gpu.py tests/test_bf16_gpu.py > gpurun_out/fast1/t.log 2>&1 || exit 1
timeout -k 10 200 python tools/probes/ds_compact_gemm.py > gpurun_out/fast1/gemm.jsonl 2>&1 || exit 1
ONLY=layer3.0,layer3.1,layer4.0,layer4.1 timeout -k 10 300 python -u tools/probes/resnet_layers.py > gpurun_out/fast1/layers_on.jsonl 2>&1 || exit 1
ONLY=layer3.0,layer3.1,layer4.0,layer4.1 DTFX_CONV_F1=0 timeout -k 10 300 python -u tools/probes/resnet_layers.py > gpurun_out/fast1/layers_off.jsonl 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/fast1/on_$r.json 2>/dev/null || exit 1
  DTFX_CONV_F1=0 timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/fast1/off_$r.json 2>/dev/null || exit 1
done
echo done
