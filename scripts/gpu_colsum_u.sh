#!/bin/bash
# bf16 column sums with 8 rows in flight: GPU tests, the probe at the decoder bias shape.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/colsum; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -k colsum -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python tools/probes/colsum_u.py > $OUT/colsum_u.json 2>&1 || { tail -20 $OUT/colsum_u.json; exit 1; }
tail -1 $OUT/colsum_u.json
