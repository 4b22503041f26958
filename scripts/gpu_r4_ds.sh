# Round-4 A/B: layer1.0's stride-1 downsample BatchNorm apply inside its narrow data gradient
# (PRO 4) vs the separate bn_bwd apply pass; interleaved on one box
set -o pipefail
mkdir -p gpurun_out/ds
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cnn_gpu.py tests/test_resnet_gpu.py > gpurun_out/ds/t.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/ds/on_$r.json 2>/dev/null || exit 1
  DTFX_DS_PROLOGUE=0 timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/ds/off_$r.json 2>/dev/null || exit 1
done
echo done
