#!/bin/bash
# LayerNorm backward variants: GPU tests, the kernel probe at the BERT shape, and interleaved
# bench.py --model bert pairs of the knob settings given (default: generic 2 slots vs H = 768).
#   scripts/gpu_ln_slots.sh ["DTFX_LN_H768=0" "DTFX_LN_H768=1"]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ln; mkdir -p $OUT
[ $# -gt 0 ] || set -- "DTFX_LN_H768=0" "DTFX_LN_H768=1"
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -k layernorm -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python tools/probes/ln_bwd_slots.py > $OUT/ln_bwd_slots.json 2>&1 || { tail -20 $OUT/ln_bwd_slots.json; exit 1; }
tail -1 $OUT/ln_bwd_slots.json
for r in 1 2 3; do
  for cfg in "$@"; do
    env $cfg timeout -k 10 200 python bench.py --model bert > "$OUT/bert_${cfg}_$r.json" 2>&1 || exit 1
    echo "round $r $cfg $(tail -1 "$OUT/bert_${cfg}_$r.json" | cut -c 100-160)"
  done
done
