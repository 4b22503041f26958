# Round-4: with the new BERT defaults, re-measure the opt-in switches that lost beside the side stream
set -o pipefail
mkdir -p gpurun_out/bcombo3
for r in 1 2; do
  timeout -k 10 300 python bench.py --model bert > gpurun_out/bcombo3/default_$r.json 2>/dev/null || exit 1
  DTFX_GEMM_TILE192=1 timeout -k 10 300 python bench.py --model bert > gpurun_out/bcombo3/tile192_$r.json 2>/dev/null || exit 1
  DTFX_GEMM_TA8=1 timeout -k 10 300 python bench.py --model bert > gpurun_out/bcombo3/ta8_$r.json 2>/dev/null || exit 1
  DTFX_BERT_OPT_OVERLAP=1 timeout -k 10 300 python bench.py --model bert > gpurun_out/bcombo3/optov_$r.json 2>/dev/null || exit 1
done
echo done
