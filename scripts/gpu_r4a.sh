#!/bin/bash
# Round 4, first GPU pass: smoke, the changed kernels' tests, BERT fold A/B, the engine trace,
# the async-PS worker breakdown, the driver-sized MLP bench.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4a; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
echo "== tests"
timeout -k 10 700 python -u -m pytest tests/test_bert_gpu.py tests/test_bf16_gpu.py tests/test_kernels_gpu.py "tests/test_xgmi_gpu.py::test_fused_mlp_exchange_matches_allreduce_engine" "tests/test_xgmi_gpu.py::test_factor_mlp_exchange_matches_allreduce_engine" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
echo "== bert"
DTFX_BERT_FOLD=0 timeout -k 10 200 python bench.py --model bert > "$OUT/bench_bert_nofold.json" 2>&1 || { tail -5 "$OUT/bench_bert_nofold.json"; exit 1; }
timeout -k 10 200 python bench.py --model bert > "$OUT/bench_bert.json" 2>&1 || { tail -5 "$OUT/bench_bert.json"; exit 1; }
tail -1 "$OUT/bench_bert_nofold.json" | cut -c 1-200; tail -1 "$OUT/bench_bert.json" | cut -c 1-200
echo "== engine trace"
timeout -k 10 200 python tools/probes/engine_trace.py > "$OUT/engine_trace.json" 2>&1 || { tail -5 "$OUT/engine_trace.json"; exit 1; }
timeout -k 10 200 python tools/probes/engine_local_cost.py > "$OUT/engine_local_cost.json" 2>&1 || { tail -5 "$OUT/engine_local_cost.json"; exit 1; }
echo "== ps"
timeout -k 10 200 python tools/probes/ps_worker_breakdown.py --mode serial > "$OUT/ps_breakdown_serial.json" 2>&1 || exit 1
timeout -k 10 200 python tools/probes/ps_worker_breakdown.py --mode pipelined > "$OUT/ps_breakdown.json" 2>&1 || exit 1
cat "$OUT/ps_breakdown_serial.json" "$OUT/ps_breakdown.json"
timeout -k 10 200 python tools/bench_ps_async.py --num_workers 2 --steps 40000 > "$OUT/ps_async_w2.json" 2>/dev/null || exit 1
cut -c 1-200 "$OUT/ps_async_w2.json"
echo "== mlp"
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > "$OUT/bench_k20.json" 2>&1 || { tail -5 "$OUT/bench_k20.json"; exit 1; }
tail -1 "$OUT/bench_k20.json" | cut -c 1-200
