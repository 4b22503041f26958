# Round-4: BERT-base step under attention-backward / weight-gradient-stream combinations
set -o pipefail
mkdir -p gpurun_out/bcombo
for r in 1 2; do
  timeout -k 10 300 python bench.py --model bert > gpurun_out/bcombo/default_$r.json 2>/dev/null || exit 1
  DTFX_ATTN_BWD_HALF=1 timeout -k 10 300 python bench.py --model bert > gpurun_out/bcombo/half_$r.json 2>/dev/null || exit 1
  DTFX_BERT_WSTREAM=0 timeout -k 10 300 python bench.py --model bert > gpurun_out/bcombo/nows_$r.json 2>/dev/null || exit 1
  DTFX_ATTN_BWD_HALF=1 DTFX_BERT_WSTREAM=0 timeout -k 10 300 python bench.py --model bert > gpurun_out/bcombo/half_nows_$r.json 2>/dev/null || exit 1
done
echo done
