# ResNet-50 BatchNorm prologue variants: tests, then interleaved A/B benches (one box)
set -o pipefail
mkdir -p gpurun_out/pro2
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_resnet_gpu.py tests/test_cnn_gpu.py > gpurun_out/pro2/t.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/pro2/all_$r.json 2>/dev/null || exit 1
  DTFX_BN_PROLOGUE_WIDE=0 timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/pro2/nowide_$r.json 2>/dev/null || exit 1
  DTFX_BN_PROLOGUE=0 DTFX_STEM_POOL_BN=0 timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/pro2/off_$r.json 2>/dev/null || exit 1
  DTFX_STEM_POOL_BN=0 timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/pro2/nostem_$r.json 2>/dev/null || exit 1
done
echo done
