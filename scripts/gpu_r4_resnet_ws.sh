# Round-4: ResNet-50 weight gradients on a side stream (opt-in) re-measured with the final kernels
set -o pipefail
mkdir -p gpurun_out/rws
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/rws/default_$r.json 2>/dev/null || exit 1
  DTFX_RESNET_WSTREAM=1 timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/rws/ws_$r.json 2>/dev/null || exit 1
done
echo done
