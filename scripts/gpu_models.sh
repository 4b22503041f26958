#!/bin/bash
# Kernel tests + BERT / ResNet benches + BERT kernel trace (rocprofv3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT=$R/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_transformer_gpu.py tests/test_bf16_gpu.py tests/test_bert_gpu.py tests/test_cnn_gpu.py tests/test_resnet_gpu.py > "$OUT/t_models.log" 2>&1 \
  || { echo FAIL tests; tail -30 "$OUT/t_models.log"; exit 1; }
tail -2 "$OUT/t_models.log"
timeout -k 10 300 python bench.py --model bert > "$OUT/bench_bert.log" 2>&1 || { echo FAIL bert; tail -20 "$OUT/bench_bert.log"; exit 1; }
tail -1 "$OUT/bench_bert.log" | cut -c1-260
timeout -k 10 300 python bench.py --model resnet50 > "$OUT/bench_resnet.log" 2>&1 || { echo FAIL resnet; tail -20 "$OUT/bench_resnet.log"; exit 1; }
tail -1 "$OUT/bench_resnet.log" | cut -c1-260
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bprof" -o run -- \
  python "$R/bench.py" --model bert --steps 6 --warmup 3 > "$OUT/bprof.log" 2>&1 || { echo FAIL prof; tail -20 "$OUT/bprof.log"; exit 1; }
python "$R/tools/trace_by_shape.py" "$OUT/bprof/run_kernel_trace.csv" > "$OUT/bprof_shapes.txt" 2>&1; head -30 "$OUT/bprof_shapes.txt"
