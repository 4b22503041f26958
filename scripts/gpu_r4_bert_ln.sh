# Round-4: LayerNorm-backward rows per block in the (now serial) BERT step
set -o pipefail
mkdir -p gpurun_out/bln
for r in 1 2; do
  timeout -k 10 300 python bench.py --model bert > gpurun_out/bln/default_$r.json 2>/dev/null || exit 1
  DTFX_LN_RPB=32 timeout -k 10 300 python bench.py --model bert > gpurun_out/bln/rpb32_$r.json 2>/dev/null || exit 1
  DTFX_LN_RPB=128 timeout -k 10 300 python bench.py --model bert > gpurun_out/bln/rpb128_$r.json 2>/dev/null || exit 1
done
echo done
