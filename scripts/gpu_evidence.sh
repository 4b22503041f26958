#!/bin/bash
# Round evidence in one gpurun call: GPU tests, MLP bench (driver-size and long runs), BERT and
# ResNet benches, rocprofv3 kernel stats of the MLP and BERT steps.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT=$R/gpurun_out/ev; mkdir -p "$OUT"; export TMPDIR=/tmp
step() { echo "== $1"; }
# PART=1: tests + benches, PART=2: ps benches + profiles (two gpurun calls), default: all
PART=${PART:-all}
if [ "$PART" != 2 ]; then
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
step tests
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
step mlp
timeout -k 10 200 python tools/probes/k20_flush.py > "$OUT/k20_flush.json" 2>&1 || exit 1
tail -1 "$OUT/k20_flush.json"
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > "$OUT/bench_mlp_k20.json" 2>&1 || exit 1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > "$OUT/bench_mlp_k20_2.json" 2>&1 || exit 1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > "$OUT/bench_mlp_k20_3.json" 2>&1 || exit 1
timeout -k 10 200 python bench.py > "$OUT/bench_mlp.json" 2>&1 || exit 1
tail -1 "$OUT/bench_mlp_k20.json" | cut -c 1-160; tail -1 "$OUT/bench_mlp.json" | cut -c 1-160
step rehearsal
DTFX_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29655 bench.py --gpus 4 --steps 200 --warmup 20 > "$OUT/rehearsal_w4.log" 2>&1 || { tail -20 "$OUT/rehearsal_w4.log"; exit 1; }
grep -h '^{' "$OUT/rehearsal_w4.log" | cut -c 1-160
step bert
timeout -k 10 200 python bench.py --model bert > "$OUT/bench_bert.json" 2>&1 || exit 1
timeout -k 10 200 python bench.py --model bert --bert_batch 32 --seq_len 512 > "$OUT/bench_bert512.json" 2>&1 || exit 1
timeout -k 10 200 python bench.py --model bert --bert_batch 256 > "$OUT/bench_bert_b256.json" 2>&1 || exit 1
tail -1 "$OUT/bench_bert.json" | cut -c 1-180; tail -1 "$OUT/bench_bert512.json" | cut -c 1-180
step resnet
timeout -k 10 200 python bench.py --model resnet50 > "$OUT/bench_resnet.json" 2>&1 || exit 1
tail -1 "$OUT/bench_resnet.json" | cut -c 1-180
timeout -k 10 240 python -u tools/probes/resnet_layers.py > "$OUT/resnet_layers.jsonl" 2>&1 || exit 1
tail -1 "$OUT/resnet_layers.jsonl"
fi
[ "$PART" = 1 ] && exit 0
step ps_async
timeout -k 10 200 python tools/probes/ps_worker_breakdown.py > "$OUT/ps_worker_breakdown.json" 2>&1 || exit 1
timeout -k 10 200 python tools/probes/engine_local_cost.py > "$OUT/engine_local_cost.json" 2>&1 || exit 1
timeout -k 10 200 python tools/bench_ps_async.py --num_workers 2 --steps 40000 > "$OUT/ps_async_w2.json" 2>/dev/null || exit 1
timeout -k 10 200 python tools/bench_ps_async.py --num_workers 8 --steps 40000 > "$OUT/ps_async_w8.json" 2>/dev/null || exit 1
timeout -k 10 200 python tools/bench_ps_async.py --num_workers 2 --steps 40000 --ps_device gpu > "$OUT/ps_async_gpu_w2.json" 2>/dev/null || exit 1
timeout -k 10 200 python tools/bench_ps_async.py --num_workers 8 --steps 40000 --ps_device gpu > "$OUT/ps_async_gpu_w8.json" 2>/dev/null || exit 1
cut -c 1-160 "$OUT/ps_async_w2.json" "$OUT/ps_async_w8.json" "$OUT/ps_async_gpu_w2.json" "$OUT/ps_async_gpu_w8.json"
step prof
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/mprof" -o run -- python "$R/bench.py" --steps 2000 --warmup 200 > "$OUT/mprof.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bprof" -o run -- python "$R/bench.py" --model bert --steps 6 --warmup 3 > "$OUT/bprof.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rprof" -o run -- python "$R/bench.py" --model resnet50 --steps 6 --warmup 3 > "$OUT/rprof.log" 2>&1 || exit 1
python "$R/tools/prof_summary.py" "$OUT/mprof/run_kernel_stats.csv" > "$OUT/mlp_kernel_stats.txt"
python "$R/tools/prof_summary.py" "$OUT/bprof/run_kernel_stats.csv" > "$OUT/bert_kernel_stats.txt"
python "$R/tools/trace_by_shape.py" "$OUT/bprof/run_kernel_trace.csv" 40 > "$OUT/bert_kernel_shapes.txt"
python "$R/tools/prof_summary.py" "$OUT/rprof/run_kernel_stats.csv" > "$OUT/resnet_kernel_stats.txt"
python "$R/tools/trace_by_shape.py" "$OUT/rprof/run_kernel_trace.csv" 40 > "$OUT/resnet_kernel_shapes.txt"
rm -f "$OUT"/rprof/*trace.csv
rm -f "$OUT"/mprof/*trace.csv
head -4 "$OUT/mlp_kernel_stats.txt"; head -12 "$OUT/bert_kernel_shapes.txt"
