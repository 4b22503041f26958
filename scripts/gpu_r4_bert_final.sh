# Round-4: BERT with the new defaults (two-blocks-per-CU attention backward, no weight-gradient
# side stream on one GPU): tests, seq 128 / 512 / batch 256 benches
set -o pipefail
mkdir -p gpurun_out/bfinal
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py tests/test_bert_gpu.py > gpurun_out/bfinal/t.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py --model bert > gpurun_out/bfinal/bert_$r.json 2>/dev/null || exit 1
done
timeout -k 10 300 python bench.py --model bert --bert_batch 32 --seq_len 512 > gpurun_out/bfinal/bert512.json 2>/dev/null || exit 1
DTFX_BERT_WSTREAM=1 timeout -k 10 300 python bench.py --model bert --bert_batch 32 --seq_len 512 > gpurun_out/bfinal/bert512_ws.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --model bert --bert_batch 256 > gpurun_out/bfinal/bert_b256.json 2>/dev/null || exit 1
echo done
