#!/bin/bash
# Round-6 probe: K=20 region split, per-shape GEMM tile A/B, BERT tile192 A/B (hipBLASLt-free).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; OUT=gpurun_out/r6probe; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 python tools/probes/k20_split.py > $OUT/k20_split.json 2>&1 || { tail $OUT/k20_split.json; exit 1; }
cat $OUT/k20_split.json
timeout -k 10 300 python tools/gemm_cfg_ab.py --cfgs 5,6 --rounds 5 --shapes qkv_fwd,out_fwd,ffn1_fwd_gelu,ffn2_fwd,qkv_dgrad,ffn1_dgrad,ffn2_dgrad_gelu,sq8192 > $OUT/gemm_ab.jsonl 2>&1 || { tail $OUT/gemm_ab.jsonl; exit 1; }
cut -c 1-200 $OUT/gemm_ab.jsonl
for i in 1 2; do for T in 0 1; do DTFX_GEMM_TILE192=$T timeout -k 10 200 python bench.py --model bert > $OUT/bert_t192_${T}_$i.json 2>&1 || exit 1; echo t192=$T; tail -1 $OUT/bert_t192_${T}_$i.json | cut -c 1-110; done; done
