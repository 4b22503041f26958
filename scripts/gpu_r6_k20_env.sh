#!/bin/bash
# Round 6: the driver-sized MLP bench under host-side settings, interleaved on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; OUT=gpurun_out/r6k20env; mkdir -p $OUT
for r in 1 2 3 4 5; do
  for v in base devkarg0 pin spin; do
    case $v in
      base) E="" ;; devkarg0) E="HIP_FORCE_DEV_KERNARG=0" ;; pin) E="DTFX_BENCH_PIN=1" ;; spin) E="DTFX_HIP_SCHED=spin" ;;
    esac
    env $E timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $OUT/${v}_$r.json 2>&1 || { tail -5 $OUT/${v}_$r.json; exit 1; }
    echo "$v $r $(tail -1 $OUT/${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["launch"])')"
  done
done
# BERT: weight gradients on the 8-phase tile (both operands transposed) vs 128x128 split-K
for r in 1 2; do for v in base ta8 ta8s128; do
  case $v in base) E="" ;; ta8) E="DTFX_GEMM_TA8=1" ;; ta8s128) E="DTFX_GEMM_TA8=1 DTFX_GEMM_TA8_SLOTS=128" ;; esac
  env $E timeout -k 10 200 python bench.py --model bert > $OUT/bert_${v}_$r.json 2>&1 || { tail -5 $OUT/bert_${v}_$r.json; exit 1; }
  echo "bert $v $r $(tail -1 $OUT/bert_${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
