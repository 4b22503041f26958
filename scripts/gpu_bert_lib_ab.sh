#!/bin/bash
# A/B of DTFX_BERT_LIB_GEMM (QKV forward + attention-output dgrad on hipBLASLt) on one box,
# interleaved, plus the BERT GPU tests on the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lib_ab; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_bert_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2 3; do
  for v in 0 1; do
    DTFX_BERT_LIB_GEMM=$v timeout -k 10 200 python bench.py --model bert > $OUT/bert_lib${v}_$r.json 2>/dev/null || exit 1
    echo "lib=$v round=$r $(tail -1 $OUT/bert_lib${v}_$r.json | cut -c 1-120)"
  done
done
