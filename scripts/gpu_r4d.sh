#!/bin/bash
# BERT (AdamW overlap / split-K fold) and async-PS (native worker step) measurements.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4d}; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== tests"
timeout -k 10 600 python -u -m pytest tests/test_bert_gpu.py tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
echo "== bert"
DTFX_BERT_OPT_OVERLAP=0 timeout -k 10 200 python bench.py --model bert > "$OUT/bench_bert_nooverlap.json" 2>&1 || { tail -5 "$OUT/bench_bert_nooverlap.json"; exit 1; }
timeout -k 10 200 python bench.py --model bert > "$OUT/bench_bert.json" 2>&1 || { tail -5 "$OUT/bench_bert.json"; exit 1; }
DTFX_BERT_OPT_OVERLAP=0 timeout -k 10 200 python bench.py --model bert > "$OUT/bench_bert_nooverlap2.json" 2>&1 || exit 1
timeout -k 10 200 python bench.py --model bert > "$OUT/bench_bert2.json" 2>&1 || exit 1
for f in bench_bert_nooverlap bench_bert bench_bert_nooverlap2 bench_bert2; do tail -1 "$OUT/$f.json" | cut -c 80-200; done
echo "== ps"
timeout -k 10 200 python tools/probes/ps_worker_breakdown.py --mode pipelined > "$OUT/ps_breakdown.json" 2>&1 || exit 1
tail -1 "$OUT/ps_breakdown.json"
timeout -k 10 200 python tools/bench_ps_async.py --num_workers 2 --steps 40000 > "$OUT/ps_async_w2.json" 2>/dev/null || exit 1
timeout -k 10 200 python tools/bench_ps_async.py --num_workers 8 --steps 40000 > "$OUT/ps_async_w8.json" 2>/dev/null || exit 1
cut -c 1-200 "$OUT/ps_async_w2.json" "$OUT/ps_async_w8.json"
