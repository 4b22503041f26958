#!/bin/bash
# Interleaved end-to-end A/B of BERT-base (bench.py --model $MODEL, default bert) between settings:
#   bash scripts/gpu_bert_env_ab.sh "DTFX_GEMM_TA8=0" "DTFX_GEMM_TA8=1"   (ROUNDS=3, ARGS=...)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/env_ab; mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-3}); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    env $v timeout -k 10 200 python bench.py --model ${MODEL:-bert} ${ARGS:-} > $OUT/v${i}_$r.json 2>/dev/null || exit 1
    echo "[$v] round=$r $(tail -1 $OUT/v${i}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
