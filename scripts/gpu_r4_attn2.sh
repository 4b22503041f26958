# attention backward with P / dS stored transposed (8-B stores): tests, standalone, BERT
set -o pipefail
mkdir -p gpurun_out/attn2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_transformer_gpu.py tests/test_bert_gpu.py > gpurun_out/attn2/t.log 2>&1 || exit 1
timeout -k 10 120 python tools/probes/attn_one.py 20 > gpurun_out/attn2/one_default.json 2>&1 || exit 1
DTFX_ATTN_BWD_HALF=1 timeout -k 10 120 python tools/probes/attn_one.py 20 > gpurun_out/attn2/one_half.json 2>&1 || exit 1
DTFX_ATTN_BWD_PERSIST=1 timeout -k 10 120 python tools/probes/attn_one.py 20 > gpurun_out/attn2/one_persist.json 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py --model bert > gpurun_out/attn2/bert_$r.json 2>/dev/null || exit 1
done
echo done
