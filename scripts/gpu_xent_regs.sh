#!/bin/bash
# MLM cross-entropy with the row in registers: GPU tests, the kernel probe at the BERT shape,
# interleaved bench.py --model bert pairs (DTFX_XENT_REGS=0 / 1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/xent; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_bert_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python tools/probes/xent_regs.py > $OUT/xent_regs.json 2>&1 || { tail -20 $OUT/xent_regs.json; exit 1; }
tail -1 $OUT/xent_regs.json
for r in 1 2 3; do
  for v in 0 1; do
    DTFX_XENT_REGS=$v timeout -k 10 200 python bench.py --model bert > "$OUT/bert_regs${v}_$r.json" 2>&1 || exit 1
    echo "round $r regs $v $(tail -1 "$OUT/bert_regs${v}_$r.json" | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
