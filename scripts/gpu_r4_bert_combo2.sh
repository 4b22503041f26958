# Round-4: confirm BERT-base with the two-blocks-per-CU attention backward and no weight-gradient
# side stream vs the current defaults (interleaved, 3 rounds each)
set -o pipefail
mkdir -p gpurun_out/bcombo2
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --model bert > gpurun_out/bcombo2/default_$r.json 2>/dev/null || exit 1
  DTFX_ATTN_BWD_HALF=1 DTFX_BERT_WSTREAM=0 timeout -k 10 300 python bench.py --model bert > gpurun_out/bcombo2/half_nows_$r.json 2>/dev/null || exit 1
done
DTFX_ATTN_BWD_HALF=1 DTFX_BERT_WSTREAM=0 timeout -k 10 300 python bench.py --model bert --bert_batch 256 > gpurun_out/bcombo2/half_nows_b256.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --model bert --bert_batch 256 > gpurun_out/bcombo2/default_b256.json 2>/dev/null || exit 1
echo done
