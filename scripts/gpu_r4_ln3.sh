# Round-4 A/B: LayerNorm backward with 3 rows in flight per wave vs 2 (standalone sweep + BERT)
set -o pipefail
mkdir -p gpurun_out/ln3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py > gpurun_out/ln3/t.log 2>&1 || exit 1
DTFX_LN_DEPTH=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py -k "layernorm or ln" > gpurun_out/ln3/t3.log 2>&1 || exit 1
for r in 1 2; do
  for rpb in 64 32 128; do
    DTFX_LN_RPB=$rpb timeout -k 10 120 python tools/probes/ln_bwd_sweep.py > gpurun_out/ln3/d2_rpb${rpb}_$r.json 2>/dev/null || exit 1
    DTFX_LN_DEPTH=3 DTFX_LN_RPB=$rpb timeout -k 10 120 python tools/probes/ln_bwd_sweep.py > gpurun_out/ln3/d3_rpb${rpb}_$r.json 2>/dev/null || exit 1
  done
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --model bert > gpurun_out/ln3/bert_d2_$r.json 2>/dev/null || exit 1
  DTFX_LN_DEPTH=3 timeout -k 10 300 python bench.py --model bert > gpurun_out/ln3/bert_d3_$r.json 2>/dev/null || exit 1
done
echo done
