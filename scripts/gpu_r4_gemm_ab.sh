# BERT GEMM tile choices (standalone, interleaved rounds) + the MLM head logits GEMM
set -o pipefail
mkdir -p gpurun_out/gab
timeout -k 10 300 python tools/gemm_cfg_ab.py --cfgs 0,5,6 --rounds 5 --shapes qkv_fwd,out_fwd,qkv_dgrad,ffn2_dgrad_gelu,ffn1_wgrad,qkv_wgrad > gpurun_out/gab/cfg_ab.jsonl 2>&1 || exit 1
timeout -k 10 200 python tools/probes/bert_head_gemm.py > gpurun_out/gab/head.jsonl 2>&1 || exit 1
echo done
