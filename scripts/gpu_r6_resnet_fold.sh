#!/bin/bash
# Round 6: ResNet-50 split-K weight gradients folded into momentum SGD (DTFX_RESNET_FOLD,
# VERDICT r5 item 7) -- tests, interleaved A/B, launch count; BERT weight gradients on the
# 8-phase tile (DTFX_GEMM_TA8) re-checked on this round's kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; OUT=gpurun_out/r6fold; mkdir -p $OUT
R=$PWD
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_resnet_gpu.py tests/test_cnn_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2 3; do for v in 1 0; do
  DTFX_RESNET_FOLD=$v timeout -k 10 300 python bench.py --model resnet50 > $OUT/resnet_fold${v}_$r.json 2>&1 || { tail -5 $OUT/resnet_fold${v}_$r.json; exit 1; }
  echo "resnet fold=$v $r $(tail -1 $OUT/resnet_fold${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/rprof" -o run -- python "$R/bench.py" --model resnet50 --steps 6 --warmup 3 > "$R/$OUT/rprof.log" 2>&1 || { tail -20 "$R/$OUT/rprof.log"; exit 1; }
cd "$R"
python tools/prof_summary.py $OUT/rprof/run_kernel_stats.csv 9 > $OUT/resnet_kernel_stats.txt && tail -1 $OUT/resnet_kernel_stats.txt
for r in 1 2; do for v in 0 1; do
  DTFX_GEMM_TA8=$v timeout -k 10 200 python bench.py --model bert > $OUT/bert_ta8_${v}_$r.json 2>&1 || { tail -5 $OUT/bert_ta8_${v}_$r.json; exit 1; }
  echo "bert ta8=$v $r $(tail -1 $OUT/bert_ta8_${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
