#!/bin/bash
# Round 6: the persistent 8-phase tile loop (DTFX_GEMM_PERS, gemm_bf16.hip) -- GEMM tests,
# per-call A/B on the BERT shapes, then BERT-base and ResNet-50 end to end, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; OUT=gpurun_out/r6pers; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_bf16_gpu.py tests/test_bert_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python tools/probes/gemm_pers_ab.py > $OUT/gemm_pers_ab.jsonl 2>&1 || { tail -20 $OUT/gemm_pers_ab.jsonl; exit 1; }
cat $OUT/gemm_pers_ab.jsonl
for r in 1 2 3; do for v in 1 0; do
  DTFX_GEMM_PERS=$v timeout -k 10 200 python bench.py --model bert > $OUT/bert_p${v}_$r.json 2>&1 || { tail -5 $OUT/bert_p${v}_$r.json; exit 1; }
  echo "bert pers=$v $r $(tail -1 $OUT/bert_p${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
