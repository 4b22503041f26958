#!/bin/bash
# Vocabulary-wide GEMMs on the 8-phase tile: bf16 / BERT GPU tests, the decoder shapes' tile
# A/B (auto should now match cfg 5 for the logits), BERT benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dec; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_bf16_gpu.py tests/test_bert_gpu.py tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python tools/gemm_cfg_ab.py --shapes dec_fwd --cfgs 0,5 > $OUT/dec_cfg_after.jsonl 2>&1 || exit 1
tail -1 $OUT/dec_cfg_after.jsonl
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --model bert > "$OUT/bert_$r.json" 2>&1 || exit 1
  echo "bert $r $(tail -1 "$OUT/bert_$r.json" | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
