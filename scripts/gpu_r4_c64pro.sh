# Round-4 A/B: relu(bn1(c1)) formed in the 64-channel 3x3 kernel's patch staging
# (DTFX_BN_PROLOGUE_C64=1, opt-in) vs the separate bn_apply pass (default)
set -o pipefail
mkdir -p gpurun_out/c64pro
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py tests/test_resnet_gpu.py > gpurun_out/c64pro/t.log 2>&1 || exit 1
for r in 1 2 3; do
  DTFX_BN_PROLOGUE_C64=1 timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/c64pro/on_$r.json 2>/dev/null || exit 1
  DTFX_BN_PROLOGUE_C64=0 timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/c64pro/off_$r.json 2>/dev/null || exit 1
done
echo done
