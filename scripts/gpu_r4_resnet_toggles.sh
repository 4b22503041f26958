# Round-4: ResNet-50 default switches re-measured with the final kernels (each turned off alone)
set -o pipefail
mkdir -p gpurun_out/rtog
for r in 1 2; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/rtog/default_$r.json 2>/dev/null || exit 1
  for v in DTFX_CONV_WGRAD_PH8 DTFX_CONV_SPLITK DTFX_STEM_WGRAD_BN DTFX_BN_PROLOGUE_WIDE DTFX_STEM_POOL_BN; do
    env $v=0 timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/rtog/${v}_off_$r.json 2>/dev/null || exit 1
  done
done
echo done
