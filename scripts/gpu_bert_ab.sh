#!/bin/bash
# BERT-base A/B of GEMM tile / stream knobs in one gpurun session (same box), two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFGS=("DTFX_GEMM_TILE192=1 DTFX_BERT_WSTREAM=1" "DTFX_GEMM_TILE192=0 DTFX_BERT_WSTREAM=1"
      "DTFX_GEMM_TILE192=1 DTFX_BERT_WSTREAM=0" "DTFX_GEMM_TILE192=0 DTFX_BERT_WSTREAM=0")
for r in 1 2; do
  for cfg in "${CFGS[@]}"; do
    env $cfg timeout -k 10 200 python bench.py --model bert > gpurun_out/bb.log 2>&1 || exit 1
    echo "$cfg $(tail -1 gpurun_out/bb.log | cut -c 80-140)"
  done
done
